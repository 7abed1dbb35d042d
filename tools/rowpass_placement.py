#!/usr/bin/env python3
"""Development tool (not shipped, not a test): which CU each rowpass
workgroup ran on (XCC_ID / HW_ID stamped by a SATRL_PHASE_PROBE build) and
the start/end times of the grid's two halves.  Used for the round-2
phase-shifted 16-row rowpass A/B:
    python3 tools/rowpass_placement.py <probe .so> <workgroups>"""
import ctypes as C, os, sys, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
import satrl._lib as _L
_L.LIB_PATH = os.path.abspath(sys.argv[1])
from satrl.ppo import PPOLearner
from satrl.trainer import args_param
H, mb = 256, 4096
a = args_param(hidden_width=H, mini_batch_size=mb, batch_size=16 * mb, chkpt_dir="/tmp")
L = PPOLearner(a, "pursuer", use_graph=False); L.sync_w2t()
g = torch.Generator(device="cuda").manual_seed(0)
src = torch.randn((16 * mb, 32), device="cuda", generator=g)
src[:, 21:24] = -1.0 - torch.rand((16 * mb, 3), device="cuda", generator=g)
st = L.stepper(mb)
for _ in range(5): st.rowpass(src, None)
torch.cuda.synchronize()
buf = np.zeros((512, 16, 16, 2), dtype=np.uint64)
lib = _L.lib(); lib.satrl_probe_read.argtypes = [C.c_void_p]
assert lib.satrl_probe_read(buf.ctypes.data) == 0
nwg = int(sys.argv[2])
xcc = buf[:nwg, 15, 0, 0].astype(np.int64) & 0xF
hw = buf[:nwg, 15, 0, 1].astype(np.int64)
cu = (hw >> 8) & 0xF; sh = (hw >> 12) & 1; se = (hw >> 13) & 0x7
key = xcc * 1000 + se * 100 + sh * 10 + cu
from collections import defaultdict
d = defaultdict(list)
for b, k in enumerate(key): d[int(k)].append(b)
sizes = np.bincount([len(v) for v in d.values()])
print("distinct CUs", len(d), "WGs per CU histogram", sizes.tolist())
pairs = [v for v in d.values() if len(v) == 2]
diffs = np.array([abs(v[1] - v[0]) for v in pairs])
print("blockIdx distance within CU pairs: ", np.unique(diffs, return_counts=True))
print("sample", list(d.items())[:6])
b = buf[:nwg].astype(np.int64)
t0 = b[:, 0, 0, 0]
print("start realtime ticks rel: first half median", np.median(t0[:nwg//2] - t0.min()), "second half", np.median(t0[nwg//2:] - t0.min()))
print("end ticks: ", np.median(b[:nwg//2, 7, 0, 0] - t0.min()), np.median(b[nwg//2:, 7, 0, 0] - t0.min()), "max", (b[:, 7, :8, 0].max() - t0.min()))
