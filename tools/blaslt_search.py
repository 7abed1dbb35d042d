#!/usr/bin/env python3
"""Development tool (not shipped, not a test): runs tools/blaslt_search.cpp
inside a torch process, so every hipBLASLt solution of the dW2 slabs is timed
on the library copy the product uses (torch's bundled hipBLASLt).
Usage: python tools/blaslt_search.py [mb]"""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
torch.zeros(1, device="cuda")                     # HIP runtime up (torch's copy)
lib = C.CDLL(os.path.join(ROOT, "tools", "_probe", "libblaslt_search.so"))
sys.exit(lib.blaslt_search(int(sys.argv[1]) if len(sys.argv) > 1 else 4096))
