#!/usr/bin/env python3
"""Development tool (not shipped, not a test): in-graph time of one fused
minibatch step (rowpass -> dW2 -> reduce -> Adam) at H 256 (PROBE_H sets
another width) for the given minibatch sizes, replaying the update's graphs
over a 16-minibatch epoch; SATRL_LIB_PATH selects a library build.
Usage: python tools/minibatch_time.py 512 1024 2048 4096"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
from satrl.ppo import PPOLearner  # noqa: E402
from satrl.trainer import args_param  # noqa: E402

H = int(os.environ.get("PROBE_H", "256"))
for mb in [int(x) for x in sys.argv[1:]] or [4096]:
    B = 16 * mb
    a = args_param(hidden_width=H, mini_batch_size=mb, batch_size=B, chkpt_dir="/tmp")
    L = PPOLearner(a, "pursuer", graph_group=16)
    g = torch.Generator(device="cuda").manual_seed(0)
    src = torch.randn((B, 32), device="cuda", generator=g)
    src[:, 21:24] = -1.0 - torch.rand((B, 3), device="cuda", generator=g)
    st = L.stepper(mb)
    perm = torch.randperm(B, device="cuda", generator=g)
    for _ in range(3):
        st.run(src, perm)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        st.run(src, perm)
    e1.record()
    torch.cuda.synchronize()
    print(f"H {H} mb {mb:5d}: {e0.elapsed_time(e1) * 1e3 / (n * 16):7.2f} us per minibatch step "
          f"(SATRL_RP_SHORT_MB={os.environ.get('SATRL_RP_SHORT_MB', 'default')}, "
          f"SATRL_FUSED_ADAM={os.environ.get('SATRL_FUSED_ADAM', 'default')})", flush=True)
