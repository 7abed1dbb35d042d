#!/usr/bin/env python3
"""Workload for the PMC passes of tools/profile_round.sh: the product's
rowpass launch at a BASELINE shape, back to back -- satrl_ppo_rowpass_kx at
the bench configuration (argv: iters 256 4096; minibatch 4096 rows drawn by a
random permutation from a packed buffer of 16384 x 2048 transitions and
staged contiguously first, as the update's graphs do with satrl_ppo_stage;
the staging copy is not a rowpass launch), satrl_ppo_rowpass_dw2 at
configs[1] (iters 64 4096: 4096 envs x 2048 steps).
rocprofv3 --pmc counts every dispatch; summarize_profiles.py keeps the
rowpass ones."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))

from satrl.ppo import PPOLearner  # noqa: E402
from satrl.trainer import args_param  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    mb = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    rows = (16384 if H == 256 else 4096) * 2048
    a = args_param(hidden_width=H, mini_batch_size=mb, batch_size=rows, chkpt_dir="/tmp")
    L = PPOLearner(a, "pursuer", use_graph=False)
    L.sync_w2t()
    g = torch.Generator(device="cuda").manual_seed(0)
    src = torch.randn((rows, 32), device="cuda", generator=g)
    perm = torch.randperm(rows, device="cuda", generator=g)
    st = L.stepper(mb)
    for k in range(iters):
        rows_k = src.index_select(0, perm[k * mb:(k + 1) * mb])
        (st.rowpass_kx if st.kx(mb) else st.rowpass_dw2 if st.fused_dw2 else st.rowpass)(rows_k, None)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
