#!/usr/bin/env python3
"""Development tool (round 4 A/B): write variant copies of the product
ppo_kernels.hip into tools/_probe/ab4/<name>.hip by exact text substitution
(each substitution must match once), for `make variant VSRC=...`.  The
product source carries no dev knobs; a variant is the product source with
one change.  Usage: python tools/ab_variants.py [name ...]  (default: all)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ppo-rl-satellite_amd", "csrc", "ppo_kernels.hip")
OUT = os.path.join(ROOT, "tools", "_probe", "ab4")

VARIANTS = {
    # (round 4: L2 warm-up of W2 / W2T, reduce chunk counts, Adam's table load,
    # bf16x3 prefetch depth / A buffering / wave counts were measured against
    # this harness; EXPERIMENTS.md)
    "dw3s16": [("constexpr int kDw3Wgs = 256;", "constexpr int kDw3Wgs = 512;")],
    "dw3s32": [("constexpr int kDw3Wgs = 256;", "constexpr int kDw3Wgs = 1024;")],
}


def main(names):
    src = open(SRC).read()
    os.makedirs(OUT, exist_ok=True)
    for name in names or VARIANTS:
        s = src
        for a, b in VARIANTS[name]:
            if s.count(a) != 1:
                raise SystemExit(f"variant {name}: substitution matches {s.count(a)} times: {a[:60]!r}")
            s = s.replace(a, b)
        with open(os.path.join(OUT, name + ".hip"), "w") as f:
            f.write(s)
        print(name)


if __name__ == "__main__":
    main(sys.argv[1:])
