#!/usr/bin/env python3
"""Development tool (not shipped, not a test): rank the hipBLASLt dW2
solutions of a minibatch shape by the IN-GRAPH minibatch step time, where
dW2's operands arrive cold from the rowpass (back-to-back timing on warm
scratch slabs ranks tiles differently).  The fastest
candidates by the tuner's clock (satrl_ppo_dw2_lib_candidates, bitwise
repeatable ones only) are each forced in a fresh process (SATRL_DW2_ALGO,
table off) and timed with tools/minibatch_time.py.

    python tools/dw2_insitu.py [mb ...] [--top N]
"""
import ctypes as C
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))


def main():
    args = sys.argv[1:]
    top = 10
    if "--top" in args:
        top = int(args[args.index("--top") + 1])
        del args[args.index("--top"):args.index("--top") + 2]
    mbs = [int(a) for a in args] or [4096]
    import torch
    from satrl import _lib
    torch.zeros(1, device="cuda")
    lib = _lib.lib()
    for mb in mbs:
        S = 4 if mb % 4 == 0 else 1
        idx = (C.c_int * top)()
        us = (C.c_float * top)()
        n = lib.satrl_ppo_dw2_lib_candidates(256, mb, -1, S, idx, us, top)
        print(f"mb {mb}: {n} repeatable candidates (back-to-back us): "
              + ", ".join(f"{idx[k]}:{us[k]:.1f}" for k in range(max(n, 0))), flush=True)
        res = []
        for k in range(max(n, 0)):
            env = dict(os.environ, SATRL_DW2_PLANS="none", SATRL_DW2_ALGO=str(idx[k]))
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "minibatch_time.py"), str(mb)],
                                 env=env, capture_output=True, text=True, timeout=300)
            m = re.search(r"([0-9.]+) us per minibatch step", out.stdout)
            t = float(m.group(1)) if m else float("nan")
            res.append((t, idx[k], us[k]))
            print(f"  solution {idx[k]}: in-graph step {t:.2f} us (tuner {us[k]:.1f} us)", flush=True)
        res.sort()
        print(f"mb {mb}: best in-graph {res[0] if res else None}", flush=True)


if __name__ == "__main__":
    main()
