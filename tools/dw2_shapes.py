#!/usr/bin/env python3
"""Development timing (not shipped, not a test): the dW2 weight-gradient GEMM
of one minibatch (2 nets x dZ2^T @ H1, K = mb rows, H x H outputs) in the
library formulations torch.bmm can hand hipBLASLt, each captured 50 times in
one hipGraph so launch overhead is out: the current split-K layout
(z^T @ y per split), the transposed product (y^T @ z = dW2^T), and split
counts 1/2/4/8/16."""
import torch

H, mb, nets = 256, 4096, 2
g = torch.Generator(device="cuda").manual_seed(0)
z = torch.randn(nets * mb * H, device="cuda", generator=g)
y = torch.randn(nets * mb * H, device="cuda", generator=g)


def timed(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        for _ in range(reps):
            fn()
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(4):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (4 * reps)


for S in (1, 2, 4, 8, 16):
    zz = z.view(nets * S, mb // S, H)
    yy = y.view(nets * S, mb // S, H)
    out = torch.empty(nets * S, H, H, device="cuda")
    t1 = timed(lambda: torch.bmm(zz.transpose(1, 2), yy, out=out))
    t2 = timed(lambda: torch.bmm(yy.transpose(1, 2), zz, out=out))
    print(f"S={S:2d}: z^T y {t1:7.2f} us   y^T z {t2:7.2f} us", flush=True)
