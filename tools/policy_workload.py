#!/usr/bin/env python3
"""Workload for the policy-kernel MFMA pass of tools/profile_round.sh: the
rollout's fused choose_action (satrl_policy_act, both agents; argv: iters
H envs, default 40 256 16384; configs[1]: 64 4096), launched back to back with random-init (orthogonal)
pursuer and evader parameters, as in the bench's rollout."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))

from satrl.ppo import PPOLearner, policy_act  # noqa: E402
from satrl.trainer import args_param  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    a = args_param(hidden_width=H, mini_batch_size=4096, batch_size=n * 2048, chkpt_dir="/tmp")
    pursuer = PPOLearner(a, "pursuer", use_graph=False)
    evader = PPOLearner(a, "evader", use_graph=False)
    g = torch.Generator(device="cuda").manual_seed(3)
    obs = torch.randn((n, 18), device="cuda", generator=g) * 1e4
    act0, logp0, act1, logp1 = (torch.empty((n, 3), device="cuda") for _ in range(4))
    for k in range(iters):
        policy_act(H, obs, pursuer.P, evader.P, 1.6, 1234, 0, k, act0, logp0, act1, logp1)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
