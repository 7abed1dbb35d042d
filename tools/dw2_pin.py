"""Write ppo-rl-satellite_amd/satrl/dw2_plans.json: the hipBLASLt dW2
solution of every H = 256 minibatch shape the engine and its tests step
(the tuner's choice, made once on an MI355X), so later runs and processes
pin the same solution instead of re-tuning.

    python tools/dw2_pin.py [out.json]      (on the GPU box)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
os.environ["SATRL_DW2_PLANS"] = "none"          # tune every shape afresh

import ctypes as C  # noqa: E402

import torch  # noqa: E402

from satrl import _lib  # noqa: E402
from satrl.ppo import dw2_plan_info  # noqa: E402

H = 256
MBS = (64, 100, 128, 256, 512, 777, 1024, 2048, 4096)
# shapes the bench and the data-parallel modes step (mb 4096 / world): ranked IN the
# update's graphs (tools/dw2_insitu.py), where dW2's operands arrive cold from the
# rowpass -- back-to-back timing on warm scratch slabs ranks tiles differently
INSITU = (512, 1024, 2048, 4096)


def insitu_best(mb, top=6):
    import re
    import subprocess
    S = 4 if mb % 4 == 0 else 1
    lib = _lib.lib()
    idx, us = (C.c_int * top)(), (C.c_float * top)()
    n = lib.satrl_ppo_dw2_lib_candidates(H, mb, -1, S, idx, us, top)
    best = None
    for k in range(max(n, 0)):
        env = dict(os.environ, SATRL_DW2_PLANS="none", SATRL_DW2_ALGO=str(idx[k]))
        t = float("inf")
        for _ in range(2):                       # the faster of two fresh processes
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "minibatch_time.py"), str(mb)], env=env,
                                 capture_output=True, text=True, timeout=300)
            m = re.search(r"([0-9.]+) us per minibatch step", out.stdout)
            if m:
                t = min(t, float(m.group(1)))
        print(f"  mb {mb} solution {idx[k]}: in-graph {t:.2f} us", flush=True)
        if best is None or t < best[0]:
            best = (t, idx[k])
    return best


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "ppo-rl-satellite_amd", "satrl", "dw2_plans.json")
    torch.zeros(1, device="cuda")
    lib = _lib.lib()
    plans = []
    for mb in MBS:
        S = 4 if mb % 4 == 0 else 1
        for net, nets in ((-1, 2), (1, 1)):
            how = "tuner"
            if net == -1 and mb in INSITU:
                best = insitu_best(mb)
                if best is not None and best[0] < float("inf"):
                    _lib.check(lib.satrl_ppo_dw2_lib_pin(H, mb, net, S, best[1], None), "satrl_ppo_dw2_lib_pin")
                    how = f"in-graph step {best[0]:.2f} us (tools/dw2_insitu.py ranking)"
            wsb, idx = C.c_int64(), C.c_int()
            _lib.check(lib.satrl_ppo_dw2_lib_workspace(H, mb, net, S, C.byref(wsb), C.byref(idx)),
                       "satrl_ppo_dw2_lib_workspace")
            i, name = dw2_plan_info(H, mb, net, S)
            plans.append({"H": H, "mb": mb, "S": S, "nets": nets, "index": i, "kernel": name,
                          "workspace_bytes": wsb.value, "chosen_by": how})
            print(json.dumps(plans[-1]), flush=True)
    with open(out, "w") as f:
        json.dump({"note": "hipBLASLt dW2 solutions per (H, mb, S, nets), chosen on an MI355X with torch's "
                           "bundled hipBLASLt: by the in-graph minibatch step time for the bench / DP shapes, else "
                           "by the dW2 tuner (csrc/dw2_blas.cpp); pinned by satrl.ppo.dw2_pin_plan "
                           "(tools/dw2_pin.py)",
                   "torch": torch.__version__, "plans": plans}, f, indent=1)


if __name__ == "__main__":
    main()
