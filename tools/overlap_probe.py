#!/usr/bin/env python3
"""Development probe (not shipped, not a test): can the rowpass and a dW2
GEMM share the chip?  Times, eager on two streams, N rowpass launches alone,
N dW2 launches alone (independent buffers), and the two interleaved on two
streams.  If the pair takes about max(), a rowpass whose phases D/E run
beside dW2 could hide the GEMM; if about the sum, they do not co-reside."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
from satrl.ppo import FusedMinibatch, PPOLearner  # noqa: E402
from satrl.trainer import args_param  # noqa: E402

H, mb, N = 256, 4096, 200
a = args_param(hidden_width=H, mini_batch_size=mb, batch_size=16 * mb, chkpt_dir="/tmp")
L = PPOLearner(a, "pursuer", use_graph=False)
L.sync_w2t()
g = torch.Generator(device="cuda").manual_seed(0)
src = torch.randn((16 * mb, 32), device="cuda", generator=g)
src[:, 21:24] = -1.0 - torch.rand((16 * mb, 3), device="cuda", generator=g)
A = FusedMinibatch(L, mb, 16, use_graph=False)
B = FusedMinibatch(L, mb, 16, use_graph=False)
H1, dZ2 = B.rowpass(src, None)
torch.cuda.synchronize()
sA, sB = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(N):
        fn()
    e1.record(torch.cuda.current_stream())
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / N


def rp():
    A.rowpass(src, None)


def dw():
    B._dw2(H1, dZ2, mb, B.S, -1)


def both():
    cur = torch.cuda.current_stream()
    sA.wait_stream(cur)
    sB.wait_stream(cur)
    with torch.cuda.stream(sA):
        A.rowpass(src, None)
    with torch.cuda.stream(sB):
        B._dw2(H1, dZ2, mb, B.S, -1)
    cur.wait_stream(sA)
    cur.wait_stream(sB)


def both_free():
    # no join per iteration: the two streams run free, joined at the end
    with torch.cuda.stream(sA):
        A.rowpass(src, None)
    with torch.cuda.stream(sB):
        B._dw2(H1, dZ2, mb, B.S, -1)


t_rp, t_dw = timed(rp), timed(dw)
t_both = timed(both)
cur = torch.cuda.current_stream()
sA.wait_stream(cur)
sB.wait_stream(cur)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
sA.wait_event(e0)
sB.wait_event(e0)
for _ in range(N):
    both_free()
cur.wait_stream(sA)
cur.wait_stream(sB)
e1.record()
torch.cuda.synchronize()
t_free = e0.elapsed_time(e1) * 1e3 / N
print(f"rowpass alone {t_rp:.2f} us, dW2 alone {t_dw:.2f} us, sum {t_rp + t_dw:.2f}; "
      f"paired with a join per pair {t_both:.2f} us; two free-running streams {t_free:.2f} us per pair")
