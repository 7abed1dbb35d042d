#!/usr/bin/env python3
"""Development tool (not shipped, not a test): event time of the rollout's
fused choose_action (satrl_policy_act, both agents, H 256 unless PROBE_H)
on 16384 observations, back to back; SATRL_LIB_PATH selects a build."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
from satrl.ppo import PPOLearner, policy_act  # noqa: E402
from satrl.trainer import args_param  # noqa: E402

H, n = int(os.environ.get("PROBE_H", "256")), 16384
a = args_param(hidden_width=H, mini_batch_size=4096, batch_size=n * 2048, chkpt_dir="/tmp")
pursuer = PPOLearner(a, "pursuer", use_graph=False)
evader = PPOLearner(a, "evader", use_graph=False)
g = torch.Generator(device="cuda").manual_seed(3)
obs = torch.randn((n, 18), device="cuda", generator=g) * 1e4
act0, logp0, act1, logp1 = (torch.empty((n, 3), device="cuda") for _ in range(4))
for k in range(20):
    policy_act(H, obs, pursuer.P, evader.P, 1.6, 1234, 0, k, act0, logp0, act1, logp1)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for k in range(200):
    policy_act(H, obs, pursuer.P, evader.P, 1.6, 1234, 0, k, act0, logp0, act1, logp1)
e1.record()
torch.cuda.synchronize()
print(f"policy_act H {H} n {n}: {e0.elapsed_time(e1) * 1e3 / 200:7.2f} us per launch", flush=True)
