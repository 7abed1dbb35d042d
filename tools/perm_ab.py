#!/usr/bin/env python3
"""Development tool (not shipped, not a test): whole training iterations at
the bench configuration (BASELINE configs[2]: 16384 envs x 2048 steps, H 256,
mb 4096, 10 epochs) with the next update's epoch orders drawn beside the
rollout (VecTrainer.perm_prefetch) and without, alternating; iteration /
rollout / GAE / update milliseconds per setting."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
from satrl.trainer import VecTrainer, args_param  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
args = args_param(batch_size=16384 * 2048, mini_batch_size=4096, hidden_width=256, K_epochs=10, max_episode_steps=1000,
                  num_envs=16384, horizon=2048, seed=0, max_train_steps=int(3e6), chkpt_dir="/tmp")
tr = VecTrainer(args, flag=0, d_capture=15000.0)
tr.iteration()
torch.cuda.synchronize()
for r in range(reps):
    for on in (False, True):
        tr.perm_prefetch = on
        timers = {}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.iteration(timers)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        print(f"prefetch {int(on)}: iteration {ms:8.1f} ms | rollout {timers['rollout_ms'][0]:6.1f} gae {timers['gae_ms'][0]:5.1f} "
              f"update {timers['update_ms'][0]:7.1f}", flush=True)
