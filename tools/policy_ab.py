#!/usr/bin/env python3
"""Development timing: satrl_policy_act (both agents) and satrl_policy_value
at H 256 for 16k and 64k rows, on a given library build (argv[1])."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
import satrl._lib as _L  # noqa: E402

if len(sys.argv) > 1:
    _L.LIB_PATH = os.path.abspath(sys.argv[1])
from satrl.ppo import PPOLearner, policy_act, policy_value  # noqa: E402
from satrl.trainer import args_param  # noqa: E402

a = args_param(hidden_width=256, chkpt_dir="/tmp")
Lp, Le = PPOLearner(a, "pursuer", use_graph=False), PPOLearner(a, "evader", use_graph=False)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for N in (16384, 65536, 2049 * 16384):          # the last: the update's values pass over T + 1 steps
    big = N > 65536
    obs = torch.randn((N, 18), device="cuda") * 1e5
    a0, l0, a1, l1 = (torch.empty((N, 3), device="cuda") for _ in range(4)) if not big else (None,) * 4
    v = torch.empty(N, device="cuda")
    res = []
    fns = ([] if big else [lambda: policy_act(256, obs, Lp.P, Le.P, 1.6, 0, 0, 0, a0, l0, a1, l1)]) + \
          [lambda: policy_value(256, obs, Lp.P, v)]
    for fn in fns:
        reps = 3 if big else 50
        for _ in range(2 if big else 5):
            fn()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / reps)
    if big:
        print(f"{os.path.basename(_L.LIB_PATH)} N={N}: value {res[0] / 1e3:8.2f} ms")
    else:
        print(f"{os.path.basename(_L.LIB_PATH)} N={N}: act {res[0]:8.2f} us  value {res[1]:8.2f} us")
