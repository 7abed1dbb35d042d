#!/usr/bin/env python3
"""Development probe (not shipped, not a test): in-graph minibatch step of
the two per-net chains on two streams (FusedMinibatch split_chains), with the
critic chain started SATRL_CHAIN_OFFSET shader cycles behind the actor's, so
the chains run out of phase.  Usage: python tools/split_offset.py [mb] [group]
(offsets swept in-process)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
from satrl.ppo import FusedMinibatch, PPOLearner  # noqa: E402
from satrl.trainer import args_param  # noqa: E402

mb = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
G = int(sys.argv[2]) if len(sys.argv) > 2 else 64
B = 2 * G * mb
a = args_param(hidden_width=256, mini_batch_size=mb, batch_size=B, chkpt_dir="/tmp")
L = PPOLearner(a, "pursuer", graph_group=G)
g = torch.Generator(device="cuda").manual_seed(0)
src = torch.randn((B, 32), device="cuda", generator=g)
src[:, 21:24] = -1.0 - torch.rand((B, 3), device="cuda", generator=g)
perm = torch.randperm(B, device="cuda", generator=g)


def timed(st, n=5):
    for _ in range(2):
        st.run(src, perm)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        st.run(src, perm)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (n * B // mb)


fused = FusedMinibatch(L, mb, G)
print(f"mb {mb} group {G}: fused chain {timed(fused):.2f} us per minibatch step", flush=True)
for off in (0, 20000, 40000, 50000, 60000, 80000):
    os.environ["SATRL_CHAIN_OFFSET"] = str(off)
    st = FusedMinibatch(L, mb, G, split_chains=True)
    print(f"  split chains, critic offset {off:6d} cycles: {timed(st):.2f} us per minibatch step", flush=True)
print(f"fused chain again {timed(fused):.2f} us", flush=True)
