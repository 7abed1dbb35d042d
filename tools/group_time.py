#!/usr/bin/env python3
"""Development probe (not shipped, not a test): in-graph minibatch step of
the fused chain against the number of minibatches per captured hipGraph
(bench.py --graph-group).  Usage: python tools/group_time.py [mb]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
from satrl.ppo import FusedMinibatch, PPOLearner  # noqa: E402
from satrl.trainer import args_param  # noqa: E402

mb = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
B = 512 * mb
a = args_param(hidden_width=256, mini_batch_size=mb, batch_size=B, chkpt_dir="/tmp")
L = PPOLearner(a, "pursuer")
g = torch.Generator(device="cuda").manual_seed(0)
src = torch.randn((B, 32), device="cuda", generator=g)
src[:, 21:24] = -1.0 - torch.rand((B, 3), device="cuda", generator=g)
perm = torch.randperm(B, device="cuda", generator=g)
for G in (32, 64, 128, 256, 64):
    st = FusedMinibatch(L, mb, G)
    st.run(src, perm)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(2):
        st.run(src, perm)
    e1.record()
    torch.cuda.synchronize()
    print(f"mb {mb} graph group {G:4d}: {e0.elapsed_time(e1) * 1e3 / (2 * B // mb):.2f} us per minibatch step", flush=True)
    del st
