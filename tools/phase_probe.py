#!/usr/bin/env python3
"""Development tool (not shipped, not a test): per-phase cycle costs of
satrl_ppo_rowpass<256,16> from the SATRL_PHASE_PROBE build
(make -C ppo-rl-satellite_amd/csrc probe -> tools/_probe/libsatrl_probe.so),
and event timings of the four launches of one minibatch step at the bench
configuration (H 256, mb 4096, contiguous staged rows).

Stamps (ppo_kernels.hip PHASE_PROBE): 0 start, 8 gather issued, 9 S ready,
10 fc1 MFMA, 11 tanh(fc1) stored, 1 barrier, 2 fc2 MFMA (B), 3 output-layer
sums (C fwd), 12 head: out_sum/tanh/logp, 13 head: ratio..dz/dls, 14 head:
dz3s + row sums (12-14 wave 0 only), 4 loss head, 5 dZ2 + tail partials,
6 dH1 MFMA (D), 7 end (E).
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
import satrl._lib as _L  # noqa: E402

probe = len(sys.argv) > 1 and sys.argv[1].startswith("probe")
if probe:
    _L.LIB_PATH = (os.path.abspath(sys.argv[1][len("probe:"):]) if sys.argv[1].startswith("probe:")
                   else os.path.join(ROOT, "tools", "_probe", "libsatrl_probe.so"))
elif len(sys.argv) > 1 and sys.argv[1].endswith(".so"):
    _L.LIB_PATH = os.path.abspath(sys.argv[1])                # an A/B variant build
print("library:", _L.LIB_PATH)
from satrl.ppo import PPOLearner  # noqa: E402
if os.environ.get("SATRL_BLAS"):                       # dev A/B: torch's BLAS backend for the dW2 bmm
    torch.backends.cuda.preferred_blas_library(os.environ["SATRL_BLAS"])
    print("blas:", torch.backends.cuda.preferred_blas_library())
from satrl.trainer import args_param  # noqa: E402

H, mb = int(os.environ.get("PROBE_H", "256")), int(os.environ.get("PROBE_MB", "4096"))
CS = H == 256 and mb <= 512                     # the column-split short rowpass (4-wave workgroups)
NWV = 4 if CS else H // 16                      # waves per rowpass workgroup
print("H", H, "mb", mb)
a = args_param(hidden_width=H, mini_batch_size=mb, batch_size=16 * mb, chkpt_dir="/tmp")
L = PPOLearner(a, "pursuer", use_graph=bool(os.environ.get("PROBE_CHAIN")))   # chain: the graphed update
L.sync_w2t()
g = torch.Generator(device="cuda").manual_seed(0)
src = torch.randn((16 * mb, 32), device="cuda", generator=g)
src[:, 21:24] = -1.0 - torch.rand((16 * mb, 3), device="cuda", generator=g)
st = L.stepper(mb)
if os.environ.get("PROBE_CHAIN"):
    # the stamps of the last rowpass of graph-replayed minibatch steps (the
    # update's own conditions: Adam has just rewritten the weights)
    perm = torch.randperm(16 * mb, device="cuda", generator=g)
    for _ in range(3):
        st.run(src, perm)
    print("stamps: the last rowpass of graph-replayed minibatch steps")
else:
    for _ in range(5):
        st.rowpass_dw2(src, None) if st.fused_dw2 else st.rowpass(src, None)
torch.cuda.synchronize()

if probe:
    lib = _L.lib()
    buf = np.zeros((512, 16, 16, 2), dtype=np.uint64)
    lib.satrl_probe_read.argtypes = [C.c_void_p]
    assert lib.satrl_probe_read(buf.ctypes.data) == 0
    b = buf.astype(np.int64)                     # [wg][stamp][wave][realtime, shader clock]
    order = [0, 8, 9, 10, 11, 1, 2, 3, 12, 13, 14, 4, 5, 6, 7]   # 12-14: inside the loss head (wave 0)
    if CS:
        # rowpass_cs: 0 start, 8 gather, 9 S ready, 10 fc1 (16 tiles), 11 tanh + planes, 1 barrier, 2 B,
        # 3 C fwd, 12 X1 hand-off done, 13 partials in LDS, 4 head, 5 tail + planes, 14 X2 hand-off done,
        # 6 D (X2 loads included), 7 end.  Rows: per net and quarter j, waves 0..3
        order = [0, 8, 9, 10, 11, 1, 2, 3, 12, 13, 4, 5, 14, 6, 7]
        ngrp = 2 * ((mb + 15) // 16)
        nb = (ngrp + 7) // 8 * 32
        bb = np.arange(nb)
        jq, grp = (bb >> 3) & 3, (bb & 7) | ((bb >> 5) << 3)
        live = grp < ngrp
        b = b[:nb, :, :4]
        t0 = b[:, 0, :, 1].min(axis=1)
        print("per-wave timeline (rowpass_cs): shader-clock time after the workgroup's start, median over groups")
        for net in (0, 1):
            for j in range(4):
                sel = live & (grp % 2 == net) & (jq == j)
                print(f"  {'actor' if net == 0 else 'critic'} quarter {j}")
                for k in order:
                    v = b[sel, k, :, 1] - t0[sel, None]
                    print(f"    stamp {k:2d}: " + " ".join(f"{int(x):6d}" for x in np.median(v, axis=0)))
        ws0 = b[live, 0, :, 0].min(axis=1)
        en = b[live, 7, :, 0].max(axis=1)
        print("workgroup span: median %.2f us, max %.2f us; start spread %.2f us, kernel span %.2f us" %
              (np.median(en - ws0) / 100.0, (en - ws0).max() / 100.0, (ws0.max() - ws0.min()) / 100.0,
               (en.max() - ws0.min()) / 100.0))
        b = None
    if b is not None:
        b = b[:2 * (mb // 32), :, :NWV]               # the launched workgroups and waves only
        t0 = b[:, 0, :, 1].min(axis=1)               # workgroup start: its first wave's stamp 0
        print("per-wave timeline: each stamp's shader-clock time after the workgroup's start "
              "(median over workgroups), waves 0..%d; actor rows then critic rows" % (NWV - 1))
        for net, sl in (("actor", slice(0, None, 2)), ("critic", slice(1, None, 2))):
            print(f"  {net}")
            for k in order:
                v = b[sl, k, :, 1] - t0[sl, None]
                print(f"    stamp {k:2d}: " + " ".join(f"{int(x):6d}" for x in np.median(v, axis=0)))
        if os.environ.get("PROBE_RAW"):
            for wg in (0, 1, 100):
                print(f"raw wg {wg}: stamp: realtime ticks rel / clock rel (waves 0, 4, 8, 15)")
                rt0 = b[wg, 0, :, 0].min()
                ck0 = b[wg, 0, :, 1].min()
                for k in order:
                    print(f"   {k:2d}: " + "  ".join(f"{int(b[wg, k, w_, 0] - rt0):6d}/{int(b[wg, k, w_, 1] - ck0):7d}"
                                                 for w_ in sorted({0, NWV // 4, NWV // 2, NWV - 1})))
        nwg = 2 * (mb // 32)
        ws0 = b[:nwg, 0, :, 0].min(axis=1)
        en = b[:nwg, 7, :, 0].max(axis=1)
        cyc = (b[:nwg, 7, :, 1].max(axis=1) - b[:nwg, 0, :, 1].min(axis=1)).astype(np.float64)
        wall = (en - ws0).astype(np.float64) / 100e6
        print("workgroup span: median %.2f us, max %.2f us; shader clock over it (median GHz) %.3f" %
              (np.median(wall) * 1e6, wall.max() * 1e6, float(np.median(cyc / wall)) / 1e9))
        print("start spread %.2f us, end spread %.2f us, kernel span %.2f us" %
              ((ws0.max() - ws0.min()) / 100.0, (en.max() - en.min()) / 100.0, (en.max() - ws0.min()) / 100.0))

# event timings of each launch of one minibatch step
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
lib = _L.lib()
sp = _L.stream_ptr()
S = st.S
H1, dZ2 = st.rowpass(src, None)


def t(fn, n=200):
    for _ in range(5):
        fn()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


nsq = st.nsq[0]
res = {
    "rowpass": t(lambda: st.rowpass_kx(src, None) if st.kx(mb) else st.rowpass(src, None)),
    "dw2": t(lambda: st.dw2_kx(mb, S) if st.kx(mb) else st._dw2(H1, dZ2, mb, S, -1)),
    "reduce": t(lambda: lib.satrl_ppo_reduce(H, mb, -1, S, 3, _L.ptr(st.p2), st.p2.numel(), _L.ptr(st.pw1), _L.ptr(st.ptail),
                                             _L.ptr(L.G), _L.ptr(nsq), _L.ptr(L.steps), sp)),
    "adam": t(lambda: lib.satrl_ppo_adam(H, mb, -1, _L.ptr(nsq), _L.ptr(L.steps), _L.ptr(L.bct), L.bct.shape[0],
                                         _L.ptr(L.lr), 0.9, 0.999, 1e-5, 0.5, 1, _L.ptr(L.G), _L.ptr(L.P),
                                         _L.ptr(L.M), _L.ptr(L.V), _L.ptr(L.W2T), sp)),
    "step (4 launches)": t(lambda: st.step(src, None)),
}
perm = torch.randperm(16 * mb, device="cuda", generator=g)
st.run(src, perm)
torch.cuda.synchronize()
res["graph group of 16 / 16"] = t(lambda: st.run(src, perm), n=20) / 16
for k, v in res.items():
    print(f"{k:>24}: {v:8.2f} us")
