#!/usr/bin/env python3
"""Development timing: satrl_ppo_rowpass alone (H 256, mb 4096, contiguous
rows) for both nets in one launch and for one net, on a given library build
(argv[1], default the product library)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
import satrl._lib as _L  # noqa: E402

if len(sys.argv) > 1:
    _L.LIB_PATH = os.path.abspath(sys.argv[1])
from satrl.ppo import PPOLearner  # noqa: E402
from satrl.trainer import args_param  # noqa: E402

H, mb = 256, 4096
a = args_param(hidden_width=H, mini_batch_size=mb, batch_size=16 * mb, chkpt_dir="/tmp")
L = PPOLearner(a, "pursuer", use_graph=False)
L.sync_w2t()
g = torch.Generator(device="cuda").manual_seed(0)
src = torch.randn((16 * mb, 32), device="cuda", generator=g)
src[:, 21:24] = -1.0 - torch.rand((16 * mb, 3), device="cuda", generator=g)
st = L.stepper(mb)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for net in (-1, 0, 1):
    for _ in range(10):
        st.rowpass(src, None, net=net)
    e0.record()
    for _ in range(200):
        st.rowpass(src, None, net=net)
    e1.record()
    torch.cuda.synchronize()
    print(f"{os.path.basename(_L.LIB_PATH)} net {net:2d}: {e0.elapsed_time(e1) * 1e3 / 200:7.2f} us")
