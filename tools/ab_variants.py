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
    # bf16x3 prefetch depth / A buffering / wave counts, dW2 split counts were
    # measured against this harness; EXPERIMENTS.md)
    # (the pre-split fc2 image `kW2Pre`, phase B without early chunks `kPreB3`
    # and the LDS-only barrier `kLdsBar3` were knobs of the product source until
    # they were measured and rejected; build them from commit e2546b9's source:
    # make variant VSRC=<git show e2546b9:ppo-rl-satellite_amd/csrc/ppo_kernels.hip>)
    # timing probes only (wrong results): the split-bf16 fc2 without the weights' split VALU / without
    # the per-chunk A-plane LDS reads
    "t_nosplit": [("""    s8v bs[3];
    split3x8(b[t], bs);""", """    s8v bs[3];
    bs[0] = __builtin_bit_cast(s8v, b[t][0]);
    bs[1] = __builtin_bit_cast(s8v, b[t][1]);
    bs[2] = __builtin_bit_cast(s8v, b[t][0]);""")],
    # timing probe (wrong results): Adam's bias corrections as constants, no
    # dependent table load behind the step-count load
    "t_nobct": [("""  const double2 bca = bct2[ka < bct_len ? ka : bct_len - 1], bcc = bct2[kc < bct_len ? kc : bct_len - 1];""",
                 """  const double2 bca = bct2[0], bcc = bct2[1];""")],
    # dW2 (k-packed) split-K ways: about 128 / 512 workgroups instead of 256
    "kx128": [("constexpr int kKxWgs = 256;", "constexpr int kKxWgs = 128;")],
    "kx512": [("constexpr int kKxWgs = 256;", "constexpr int kKxWgs = 512;")],
    # dw2_kx LDS ring depth (slots; chunks kKxD - 1 ahead; 24 KB + pad per slot)
    "kxd4": [("constexpr int kKxD = 3; ", "constexpr int kKxD = 4; ")],
    "kxd6": [("constexpr int kKxD = 3; ", "constexpr int kKxD = 6; ")],
    # dw2_kx on 128x128 output tiles (half the plane bytes per workgroup, 32 splits)
    "kxt128": [("constexpr int kKxTW = 64;", "constexpr int kKxTW = 128;")],
    "t_noalds": [("""    } else {
      a3_chunk<LDP, PS, RT>(ap + 32 * c, aa[0]);
    }""", """    } else {
      if (c == 0) a3_chunk<LDP, PS, RT>(ap, aa[0]);
    }""")],
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
