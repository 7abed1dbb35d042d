#!/usr/bin/env python3
"""Workloads for the env-kernel profile passes of tools/profile_round.sh.

    env_workload.py [iters]            mid-episode: satenv step_kernel_wide<autoreset> on 16384 envs
                                       (the bench configuration), 256 untimed steps of U(-1.6,1.6)
                                       actions so episodes are mid-flight, then `iters` profiled steps
                                       (the PMC passes take the last `iters` dispatches)
    env_workload.py sweep [iters]      the same mid-episode protocol at 4096, 16384 and 65536 envs, one
                                       after the other (kernel trace split by grid size)
    env_workload.py rollout [iters]    the training rollout alone: VecTrainer.collect() at 16384 envs,
                                       hidden 256 (both agents' policy kernel -> env step, hipGraph
                                       chunks), `iters` rollouts of 2048 steps after one warm-up: every
                                       step_kernel_wide dispatch of the process is an in-rollout launch
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))

from satrl.env import VecSatellites  # noqa: E402


def mid_episode(n, iters, seed=7):
    g = torch.Generator(device="cuda").manual_seed(seed)
    env = VecSatellites(n, d_capture=15000.0, max_episode_steps=1000)
    env.reset(0)
    acts = (torch.rand((64, 2, n, 3), device="cuda", generator=g) * 3.2 - 1.6).contiguous()
    obs = torch.empty((n, 18), dtype=torch.float32, device="cuda")
    rew = torch.empty(n, dtype=torch.float32, device="cuda")
    dn = torch.empty(n, dtype=torch.uint8, device="cuda")
    for k in range(256 + iters):
        env.step_autoreset(acts[k % 64, 0], acts[k % 64, 1], obs, rew, dn)
    torch.cuda.synchronize()


def rollout(iters):
    from satrl.trainer import VecTrainer, args_param
    n, T = 16384, 2048
    args = args_param(batch_size=n * T, mini_batch_size=4096, hidden_width=256, K_epochs=1, max_episode_steps=1000,
                      num_envs=n, horizon=T, seed=0, max_train_steps=int(3e6), chkpt_dir="/tmp")
    tr = VecTrainer(args, flag=0, d_capture=15000.0)
    for _ in range(1 + iters):
        tr.collect()
        tr.buf.obs[0].copy_(tr.buf.obs[T])
    torch.cuda.synchronize()


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].isdigit() else "mid"
    rest = [a for a in sys.argv[1:] if a.isdigit()]
    iters = int(rest[0]) if rest else (1 if mode == "rollout" else 40)
    if mode == "mid":
        mid_episode(16384, iters)
    elif mode == "sweep":
        for n in (4096, 16384, 65536):
            mid_episode(n, iters)
    elif mode == "rollout":
        rollout(iters)
    else:
        raise SystemExit(f"unknown mode {mode}")
    print("ok")


if __name__ == "__main__":
    main()
