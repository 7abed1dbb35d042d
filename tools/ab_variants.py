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
    # (round 4's L2 warm-up of W2 / W2T, reduce chunk counts and Adam's table
    # load were measured against this harness; EXPERIMENTS.md)
    # the bf16x3 fc2 products: B prefetch distance / A buffering
    "b3_d3": [("constexpr int kBPD3 = 2;", "constexpr int kBPD3 = 3;")],
    "b3_d4a1": [("constexpr int kBPD3 = 2;", "constexpr int kBPD3 = 4;"),
                ("constexpr int kADB3 = 2;", "constexpr int kADB3 = 1;")],
    "b3_d6a1": [("constexpr int kBPD3 = 2;", "constexpr int kBPD3 = 6;"),
                ("constexpr int kADB3 = 2;", "constexpr int kADB3 = 1;")],
    "b3_d2a1": [("constexpr int kADB3 = 2;", "constexpr int kADB3 = 1;")],
    # 8 waves per H 256 workgroup (2 column tiles each): half the A-plane LDS reads
    "nw8": [("constexpr int kNW256 = 16;", "constexpr int kNW256 = 8;")],
    "nw8a1": [("constexpr int kNW256 = 16;", "constexpr int kNW256 = 8;"),
              ("constexpr int kADB3 = 2;", "constexpr int kADB3 = 1;")],
    "pol8": [("constexpr int kPolNW = 16;", "constexpr int kPolNW = 8;")],
    "pol8a1": [("constexpr int kPolNW = 16;", "constexpr int kPolNW = 8;"),
               ("constexpr int kADB3 = 2;", "constexpr int kADB3 = 1;")],
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
