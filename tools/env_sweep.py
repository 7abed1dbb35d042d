#!/usr/bin/env python3
"""Development timing: the env step kernel (autoreset) at 4k/16k/64k envs,
mid-episode (256 untimed steps of U(-1.6,1.6) actions first), as bench.py's
sweep; plus the same from fresh resets (first 64 steps).  argv: step kernels
to time, as kind:envs_per_workgroup[:solve_waves] (satenv_set_step_kernel,
satenv_set_solve_waves; 0 = by occupancy), default 2:64:0.  SATRL_LIB_PATH
selects a library build."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
from satrl.env import VecSatellites  # noqa: E402

e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
g = torch.Generator(device="cuda").manual_seed(7)
kinds = [tuple(int(x) for x in (a + ":0").split(":")[:3]) for a in sys.argv[1:]] or [(2, 64, 0)]
tag = os.path.basename(os.environ.get("SATRL_LIB_PATH", "product"))
for n, (kind, wide, qw) in [(n, kw) for n in (4096, 16384, 65536) for kw in kinds]:
    env = VecSatellites(n, d_capture=15000.0, max_episode_steps=1000)
    env.set_step_kernel(kind, wide)
    if hasattr(env, "set_solve_waves"):
        try:
            env.set_solve_waves(qw)
        except Exception:                     # (a library without the queue)
            pass
    env.reset(0)
    acts = (torch.rand((64, 2, n, 3), device="cuda", generator=g) * 3.2 - 1.6).contiguous()
    o = torch.empty((n, 18), dtype=torch.float32, device="cuda")
    r = torch.empty(n, dtype=torch.float32, device="cuda")
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    e0.record()
    for k in range(64):
        env.step_autoreset(acts[k, 0], acts[k, 1], o, r, d)
    e1.record()
    torch.cuda.synchronize()
    fresh = e0.elapsed_time(e1) * 1e3 / 64
    for k in range(192):
        env.step_autoreset(acts[k % 64, 0], acts[k % 64, 1], o, r, d)
    e0.record()
    for k in range(200):
        env.step_autoreset(acts[k % 64, 0], acts[k % 64, 1], o, r, d)
    e1.record()
    torch.cuda.synchronize()
    mid = e0.elapsed_time(e1) * 1e3 / 200
    print(f"[{tag}] n={n:6d} kernel {kind}:{wide:2d}:{qw}  fresh {fresh:7.2f} us  mid-episode {mid:7.2f} us  "
          f"({n / mid * 1e-3:.3f} G env-steps/s)", flush=True)
