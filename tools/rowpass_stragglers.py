#!/usr/bin/env python3
"""Development tool (not shipped, not a test): which rowpass workgroups end
last, and whether it is the same CUs / XCDs launch after launch.  Uses the
SATRL_PHASE_PROBE build (make -C ppo-rl-satellite_amd/csrc probe): per
workgroup the placement stamp (XCC_ID, HW_ID) and every wave's start / end
realtime stamps (100 MHz).
    python3 tools/rowpass_stragglers.py [launches]"""
import ctypes as C
import os
import sys
from collections import defaultdict

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
import satrl._lib as _L  # noqa: E402
_L.LIB_PATH = os.path.join(ROOT, "tools", "_probe", "libsatrl_probe.so")
from satrl.ppo import PPOLearner  # noqa: E402
from satrl.trainer import args_param  # noqa: E402

H, mb = 256, 4096
nwg = 2 * mb // 32
a = args_param(hidden_width=H, mini_batch_size=mb, batch_size=16 * mb, chkpt_dir="/tmp")
L = PPOLearner(a, "pursuer", use_graph=False)
L.sync_w2t()
g = torch.Generator(device="cuda").manual_seed(0)
src = torch.randn((16 * mb, 32), device="cuda", generator=g)
src[:, 21:24] = -1.0 - torch.rand((16 * mb, 3), device="cuda", generator=g)
st = L.stepper(mb)
lib = _L.lib()
lib.satrl_probe_read.argtypes = [C.c_void_p]
for _ in range(5):
    st.rowpass(src, None)
torch.cuda.synchronize()
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 6
ends, keys = [], None
for r in range(runs):
    st.rowpass(src, None)
    torch.cuda.synchronize()
    buf = np.zeros((512, 16, 16, 2), dtype=np.uint64)
    assert lib.satrl_probe_read(buf.ctypes.data) == 0
    b = buf[:nwg].astype(np.int64)
    start = b[:, 0, :, 0].min(axis=1)
    end = b[:, 7, :, 0].max(axis=1)
    t0 = start.min()
    ends.append((end - t0) / 100.0)                       # us after the kernel's first wave started
    xcc = b[:, 15, 0, 0] & 0xF
    hw = b[:, 15, 0, 1]
    keys = xcc * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 10 + ((hw >> 8) & 0xF)
    if r == 0:
        print("launch 0: end after first start, us: median %.2f p90 %.2f max %.2f" %
              (np.median(ends[-1]), np.percentile(ends[-1], 90), ends[-1].max()))
        for net, nm in ((0, "actor"), (1, "critic")):
            e = ends[-1][net::2]
            print(f"  {nm}: median {np.median(e):.2f} max {e.max():.2f}")
        byx = defaultdict(list)
        for wgi in range(nwg):
            byx[int(xcc[wgi])].append(ends[-1][wgi])
        print("  by XCC: " + "  ".join(f"{k}: {np.median(v):.2f}/{max(v):.2f}" for k, v in sorted(byx.items())))
E = np.array(ends)                                          # [runs][nwg]
rank = np.argsort(np.argsort(-E, axis=1), axis=1)           # 0 = last to end
slow = (rank < 16).mean(axis=0)                             # how often each WG is among the 16 last
print("launch-to-launch: per-WG end correlation between consecutive launches:",
      " ".join(f"{np.corrcoef(E[i], E[i + 1])[0, 1]:.2f}" for i in range(runs - 1)))
top = np.argsort(-slow)[:12]
print("WGs most often among the 16 last (blockIdx, net, XCC/SE/SH/CU key, fraction):")
print("  " + "  ".join(f"{w}:{w & 1}:{int(keys[w])}:{slow[w]:.2f}" for w in top))
print("kernel span per launch, us:", " ".join(f"{e.max():.2f}" for e in E))
