#!/usr/bin/env python3
"""Workload for the post-rowpass PMC passes of tools/profile_round.sh: whole
minibatch steps (rowpass_kx -> dw2_kx -> reduce -> Adam) at the bench
configuration (H 256, mb 4096, both nets), eager so every kernel is its own
dispatch.  summarize_profiles.py keeps the dW2 / reduce / Adam dispatches."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))

from satrl.ppo import PPOLearner  # noqa: E402
from satrl.trainer import args_param  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    H, mb = 256, 4096
    a = args_param(hidden_width=H, mini_batch_size=mb, batch_size=16 * mb, chkpt_dir="/tmp")
    L = PPOLearner(a, "pursuer", use_graph=False)
    L.sync_w2t()
    g = torch.Generator(device="cuda").manual_seed(0)
    src = torch.randn((16 * mb, 32), device="cuda", generator=g)
    src[:, 21:24] = -1.0 - torch.rand((16 * mb, 3), device="cuda", generator=g)
    st = L.stepper(mb)
    for k in range(iters):
        st.step(src[(k % 16) * mb:(k % 16 + 1) * mb], None)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
