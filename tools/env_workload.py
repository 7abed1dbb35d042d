#!/usr/bin/env python3
"""Workload for the env-kernel PMC passes of tools/profile_round.sh:
satenv step_kernel<autoreset> on 16384 envs (the bench configuration), 256
untimed steps with U(-1.6,1.6) actions so episodes are mid-flight, then N
profiled steps."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))

from satrl.env import VecSatellites  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    n = 16384
    g = torch.Generator(device="cuda").manual_seed(7)
    env = VecSatellites(n, d_capture=15000.0, max_episode_steps=1000)
    env.reset(0)
    acts = (torch.rand((64, 2, n, 3), device="cuda", generator=g) * 3.2 - 1.6).contiguous()
    obs = torch.empty((n, 18), dtype=torch.float32, device="cuda")
    rew = torch.empty(n, dtype=torch.float32, device="cuda")
    dn = torch.empty(n, dtype=torch.uint8, device="cuda")
    for k in range(256 + iters):
        env.step_autoreset(acts[k % 64, 0], acts[k % 64, 1], obs, rew, dn)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
