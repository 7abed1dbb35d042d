#!/usr/bin/env python3
"""Development timing (not shipped, not a test): the dW2 GEMM (2 nets x S=4
split-K slabs of 1024 rows, H 256) with its operands stored row-major per
minibatch row ([rows][H], how the rowpass writes H1 / dZ2 today) against
K-contiguous ([H][rows], a transposed store), through torch.bmm on
hipBLASLt, 50 launches captured in one hipGraph."""
import torch

torch.backends.cuda.preferred_blas_library("hipblaslt")
H, mb, S = 256, 4096, 4
B, K = 2 * S, mb // S
g = torch.Generator(device="cuda").manual_seed(0)
z = torch.randn((B, K, H), device="cuda", generator=g)
y = torch.randn((B, K, H), device="cuda", generator=g)
zt, yt = z.transpose(1, 2).contiguous(), y.transpose(1, 2).contiguous()
out = torch.empty((B, H, H), device="cuda")
forms = {
    "row-major [rows][H] (today): z^T y": lambda: torch.bmm(z.transpose(1, 2), y, out=out),
    "K-contiguous [H][rows]: zt yt^T": lambda: torch.bmm(zt, yt.transpose(1, 2), out=out),
    "mixed: zt y": lambda: torch.bmm(zt, y, out=out),
    "mixed: z^T yt^T": lambda: torch.bmm(z.transpose(1, 2), yt.transpose(1, 2), out=out),
}
ref = torch.bmm(z.transpose(1, 2).double(), y.double())
for name, fn in forms.items():
    fn()
    torch.cuda.synchronize()
    err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(50):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:40s} {e0.elapsed_time(e1) * 1e3 / 250:7.2f} us  (rel err {err:.1e})", flush=True)
