#!/usr/bin/env python3
"""Development tool: the kernel timeline of graph-replayed minibatch steps.

  python tools/step_timeline.py run          workload (under rocprofv3 --kernel-trace)
  python tools/step_timeline.py parse CSV    per-kernel durations and the gaps
                                             between consecutive kernels (us)
"""
import csv
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run():
    import torch
    sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
    from satrl.ppo import PPOLearner
    from satrl.trainer import args_param
    H, mb = int(os.environ.get("PROBE_H", "256")), int(os.environ.get("PROBE_MB", "4096"))
    a = args_param(hidden_width=H, mini_batch_size=mb, batch_size=16 * mb, chkpt_dir="/tmp")
    L = PPOLearner(a, "pursuer")
    L.sync_w2t()
    g = torch.Generator(device="cuda").manual_seed(0)
    src = torch.randn((16 * mb, 32), device="cuda", generator=g)
    src[:, 21:24] = -1.0 - torch.rand((16 * mb, 3), device="cuda", generator=g)
    st = L.stepper(mb)
    perm = torch.randperm(16 * mb, device="cuda", generator=g)
    for _ in range(int(os.environ.get("REPS", "20"))):
        st.run(src, perm)
    torch.cuda.synchronize()
    print("ok")


def short(name):
    if "rowpass" in name and "true, true>" in name.replace(";", ","):
        return "rowpass_adam"
    for k in ("rowpass", "reduce_kernel", "reduce_apply_kernel<true", "reduce_apply_kernel<false", "adam_kernel",
              "steps_advance", "dw2_kernel", "Cijk", "gather", "copy"):
        if k in name:
            return k
    return name[:40]


def parse(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    dur, gap = defaultdict(list), defaultdict(list)
    for i, (s, e, n) in enumerate(rows):
        dur[n].append((e - s) / 1e3)
        if i:
            ps, pe, pn = rows[i - 1]
            g = (s - pe) / 1e3
            if g < 50:
                gap[(pn, n)].append(g)
    med = lambda v: sorted(v)[len(v) // 2]
    print("kernel durations (median us, n):")
    for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n:>16}: {med(v):8.2f}  ({len(v)})")
    print("gaps end(prev) -> start(next) (median us, n):")
    for (a, b), v in sorted(gap.items(), key=lambda kv: -len(kv[1])):
        print(f"  {a:>16} -> {b:<16}: {med(v):6.2f}  ({len(v)})")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(sys.argv[2])
