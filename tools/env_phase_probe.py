#!/usr/bin/env python3
"""Development tool (not shipped, not a test): per-phase cycles of
step_kernel_wide<autoreset, 64> from the SATENV_PHASE_PROBE build (make -C
ppo-rl-satellite_amd/csrc probe -> tools/_probe/libsatrl_probe.so), 16384
envs mid-episode (256 untimed steps of U(-1.6, 1.6) actions first).

Stamps (satenv_kernels.hip ENV_PROBE, per wave): 0 start, 1 phase I done
(step_begin), 2 II (elements | reward terms), 3 III (set-ups), 4 IV (solves),
5 after IV's barrier, 6 end (V: finish + write-back)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
import satrl._lib as _L  # noqa: E402

_L.LIB_PATH = os.path.join(ROOT, "tools", "_probe", "libsatrl_probe.so")
from satrl.env import VecSatellites  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
g = torch.Generator(device="cuda").manual_seed(7)
env = VecSatellites(n, d_capture=15000.0, max_episode_steps=1000)
env.reset(0)
acts = (torch.rand((64, 2, n, 3), device="cuda", generator=g) * 3.2 - 1.6).contiguous()
o = torch.empty((n, 18), dtype=torch.float32, device="cuda")
r = torch.empty(n, dtype=torch.float32, device="cuda")
d = torch.empty(n, dtype=torch.uint8, device="cuda")
for k in range(256):
    env.step_autoreset(acts[k % 64, 0], acts[k % 64, 1], o, r, d)
torch.cuda.synchronize()
lib = _L.lib()
lib.satenv_probe_read.argtypes = [C.c_void_p]
buf = np.zeros((1024, 8, 4), dtype=np.uint64)
assert lib.satenv_probe_read(buf.ctypes.data) == 0
nwg = min(1024, (n + 63) // 64)
b = buf[:nwg].astype(np.int64)
names = ["I step_begin", "II elements|reward", "III set-ups", "IV solves", "IV barrier", "V finish"]
print(f"n={n}: phase cycles per wave (median over workgroups; wave 0 | 1 | 2 | 3)")
for k in range(6):
    dd = b[:, k + 1, :] - b[:, k, :]
    print(f"  {names[k]:>20}: " + " | ".join(f"{int(np.median(dd[:, w])):7d}" for w in range(4)))
tot = b[:, 6, 0] - b[:, 0, 0]
print(f"  {'total (wave 0)':>20}: {int(np.median(tot)):7d}  max {int(tot.max())}")
