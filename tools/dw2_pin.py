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


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "ppo-rl-satellite_amd", "satrl", "dw2_plans.json")
    torch.zeros(1, device="cuda")
    lib = _lib.lib()
    plans = []
    for mb in MBS:
        S = 4 if mb % 4 == 0 else 1
        for net, nets in ((-1, 2), (1, 1)):
            wsb, idx = C.c_int64(), C.c_int()
            _lib.check(lib.satrl_ppo_dw2_lib_workspace(H, mb, net, S, C.byref(wsb), C.byref(idx)),
                       "satrl_ppo_dw2_lib_workspace")
            i, name = dw2_plan_info(H, mb, net, S)
            plans.append({"H": H, "mb": mb, "S": S, "nets": nets, "index": i, "kernel": name,
                          "workspace_bytes": wsb.value})
            print(json.dumps(plans[-1]), flush=True)
    with open(out, "w") as f:
        json.dump({"note": "hipBLASLt dW2 solutions per (H, mb, S, nets), chosen by the dW2 tuner "
                           "(csrc/dw2_blas.cpp) on an MI355X with torch's bundled hipBLASLt; pinned by "
                           "satrl.ppo.dw2_pin_plan (tools/dw2_pin.py)",
                   "torch": torch.__version__, "plans": plans}, f, indent=1)


if __name__ == "__main__":
    main()
