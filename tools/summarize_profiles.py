#!/usr/bin/env python3
"""Turns rocprofv3 CSV output (tools/profile_round.sh) into the committed
summaries under profiles/: the kernel-stats table of the bench command and
the per-launch HBM traffic of the product's rowpass (H 256: rowpass_kx; H 64,
suffix _h64: rowpass_dw2) from the FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md "HBM": FETCH_SIZE reports half the
bytes of 16-B-per-lane reads on gfx950 -> x2; WRITE_SIZE exact; both in KB)."""
import csv
import json
import os
import sys


def kernel_stats(path, out):
    rows = list(csv.DictReader(open(path)))
    with open(out, "w") as f:
        f.write("name,calls,total_ns,avg_ns,min_ns,max_ns,percent\n")
        for r in rows:
            name = r["Name"].replace(",", ";")
            f.write(f'"{name}",{r["Calls"]},{r["TotalDurationNs"]},{r["AverageNs"]},{r["MinNs"]},{r["MaxNs"]},'
                    f'{r["Percentage"]}\n')
    return rows


def pmc_per_dispatch(path, kernel_sub, counter, last=None):
    per = {}
    for r in csv.DictReader(open(path)):
        if kernel_sub in r["Kernel_Name"] and r["Counter_Name"] == counter:
            k = int(r["Dispatch_Id"])
            per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
    keys = sorted(per)
    if last is not None:
        keys = keys[-last:]
    vals = sorted(per[k] for k in keys)
    return vals[len(vals) // 2] if vals else None, len(vals)


def main():
    d = sys.argv[1]          # gpurun_out/<run>
    tag = sys.argv[2]        # e.g. r1
    prof = sys.argv[3] if len(sys.argv) > 3 else os.path.join(d, "profiles")
    os.makedirs(prof, exist_ok=True)
    ks = os.path.join(d, "bench", "run_kernel_stats.csv")
    if os.path.exists(ks):
        kernel_stats(ks, os.path.join(prof, f"{tag}_bench_kernel_stats.csv"))
    ks = os.path.join(d, "bench_configs1", "run_kernel_stats.csv")      # BASELINE configs[1]'s bench command
    if os.path.exists(ks):
        kernel_stats(ks, os.path.join(prof, f"{tag}_bench_configs1_kernel_stats.csv"))
    for sfx, H in (("", 256), ("_h64", 64)):
        rowpass_summaries(d, tag, prof, sfx, H)
    sf = os.path.join(d, "pmc_step_fetch", "run_counter_collection.csv")
    sw = os.path.join(d, "pmc_step_write", "run_counter_collection.csv")
    sm = os.path.join(d, "pmc_step_mfma", "run_counter_collection.csv")
    if os.path.exists(sf) and os.path.exists(sw) and os.path.exists(sm):
        # the post-rowpass chain per launch: HBM bytes (FETCH x2 + WRITE) against
        # the algorithmic bytes, and matrix-core busy cycles (dW2 only has MFMA work)
        # the product's dW2 at this shape: dw2_kx_w1_kernel (k-packed bf16 planes, 8
        # splits, with the reduce's W1 / tail regions: their slabs in, G's parts out);
        # reduce_kernel then sums the W2 region only
        kx = True
        H, mb, S, nwg = 256, 4096, 8, 128
        tot = 2 * H * H + 2 * H * 20 + 6 * H + 12            # flat layout incl. pads (satrl_ppo_layout)
        w1t = (nwg * 2 * H * 20 + nwg * (6 * H + 12)) * 4 + (2 * H * 20 + 6 * H + 12) * 4
        dw2 = "dw2_kx_w1_kernel"
        alg = {dw2: (2 * 2 * 3 * mb * H * 2 if kx else 2 * 2 * mb * H * 4) + 2 * S * H * H * 4 + w1t,
               "reduce_kernel": 2 * S * H * H * 4 + 2 * H * H * 4,
               "adam_kernel": 4 * tot * 4 + 3 * tot * 4 + 2 * H * H * (6 if kx else 4)}
        chain = {}
        for sub in (dw2, "reduce_kernel", "adam_kernel"):
            f_kb, nf = pmc_per_dispatch(sf, sub, "FETCH_SIZE")
            w_kb, nw = pmc_per_dispatch(sw, sub, "WRITE_SIZE")
            busy, nb = pmc_per_dispatch(sm, sub, "SQ_VALU_MFMA_BUSY_CYCLES")
            grbm, ng = pmc_per_dispatch(sm, sub, "GRBM_GUI_ACTIVE")
            hbm = (2 * f_kb + w_kb) * 1024.0 if f_kb is not None and w_kb is not None else None
            chain[sub] = {"dispatches": [nf, nw, nb, ng], "FETCH_SIZE_kB_median": f_kb, "WRITE_SIZE_kB_median": w_kb,
                          "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": alg[sub],
                          "traffic_over_algorithmic": hbm / alg[sub] if hbm else None,
                          "SQ_VALU_MFMA_BUSY_CYCLES_median": busy, "GRBM_GUI_ACTIVE_median": grbm,
                          "mfma_busy_frac_dispatch_window": busy / (grbm / 8.0 * 1024) if busy and grbm else None}
        res = {"kernels": chain, "hidden": H, "minibatch": mb, "dw2_splits": S,
               "correction": "FETCH_SIZE x2 (gfx950 16-B/lane reads), WRITE_SIZE x1; kB = 1024 B",
               "definition": "per-dispatch medians; dw2_kx_w1_kernel = the split-bf16 dW2 on the rowpass's k-packed "
                             "planes (1.07 GFLOP per launch, f32-equivalent) with the reduce's W1 / tail regions; "
                             "mfma_busy_frac as in the rowpass summary, over the --pmc dispatch window (a lower "
                             "bound for short dispatches)",
               "workload": "tools/step_workload.py (eager minibatch steps)"}
        with open(os.path.join(prof, f"{tag}_chain_pmc.json"), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res))
    for sfx, H, n in (("", 256, 16384), ("_h64", 64, 4096)):
        policy_summary(d, tag, prof, sfx, H, n)
    fetch = os.path.join(d, "pmc_env_fetch", "run_counter_collection.csv")
    write = os.path.join(d, "pmc_env_write", "run_counter_collection.csv")
    if os.path.exists(fetch) and os.path.exists(write):
        # the last 40 dispatches are the profiled mid-episode steps (256 warm-up steps first)
        f_kb, nf = pmc_per_dispatch(fetch, "step_kernel", "FETCH_SIZE", last=40)
        w_kb, nw = pmc_per_dispatch(write, "step_kernel", "WRITE_SIZE", last=40)
        n = 16384
        res = {"kernel": "satenv step_kernel_wide<true, 64>", "num_envs": n, "dispatches": [nf, nw],
               "FETCH_SIZE_kB_median": f_kb, "WRITE_SIZE_kB_median": w_kb,
               "fetch_bytes_per_env_raw": f_kb * 1024.0 / n, "write_bytes_per_env": w_kb * 1024.0 / n,
               "hbm_bytes_per_launch": (2 * f_kb + w_kb) * 1024.0,
               "correction": "FETCH_SIZE x2 as for 16-B/lane reads (the kernel's f64 plane loads are 8 B/lane, "
                             "uncalibrated per MI355X_MICROARCH.md; raw per-env fetch bytes kept beside), "
                             "WRITE_SIZE x1; kB = 1024 B",
               "workload": "tools/env_workload.py"}
        with open(os.path.join(prof, f"{tag}_env_pmc.json"), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res))
    env_extra(d, tag, prof)


MFMA_DEF = ("mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the fraction of "
            "SIMD-cycles of the dispatch window in which the matrix core was busy, at the clock the chip ran "
            "(roofline.frac prices against the 2.4 GHz peak instead). The window of a ~10-30 us dispatch under "
            "--pmc includes the profiler's per-dispatch set-up (MI355X_MICROARCH.md: GRBM quotients read high below "
            "~0.3 ms), so this is a lower bound; busy_over_expected = 1 shows the counter equals the MFMAs' busy "
            "cycles (32 per f32 16x16x4, 16 per bf16 16x16x32)")


def rowpass_mfma_counts(H, mb):
    """(f32 16x16x4, bf16 16x16x32) MFMA instructions of one product rowpass
    launch over both nets.  H 256 (rowpass_kx, 32-row blocks of 16 waves, one
    16-column tile each): fc1 fwd + [dW1|db1] 32 f32 per wave (K padded to 32),
    fc2 fwd + dH1 as split-bf16 8 chunks x 2 row tiles x 6 products x 2 phases
    = 192 per wave.  H 64 (rowpass_dw2, 32-row blocks of 4 waves): fc1 16, fc2
    and dH1 2 chunks x 16 each, [dW1|db1] 16, the fused dW2 partial 8 x 4 =
    32: 128 f32 per wave."""
    wgs = 2 * ((mb + 31) // 32)
    if H == 256:
        return wgs * 16 * 32, wgs * 16 * 192
    return wgs * 4 * 128, 0


def rowpass_summaries(d, tag, prof, sfx, H):
    mb = 4096
    kernel = "rowpass_kernel<256, 16, 32, kx>" if H == 256 else "rowpass_kernel<64, 4, 32, fused dW2>"
    fetch = os.path.join(d, "pmc_fetch" + sfx, "run_counter_collection.csv")
    write = os.path.join(d, "pmc_write" + sfx, "run_counter_collection.csv")
    if os.path.exists(fetch) and os.path.exists(write):
        f_kb, nf = pmc_per_dispatch(fetch, "rowpass_kernel", "FETCH_SIZE")
        w_kb, nw = pmc_per_dispatch(write, "rowpass_kernel", "WRITE_SIZE")
        res = {"kernel": kernel, "hidden": H, "minibatch": mb,
               "dispatches": [nf, nw], "FETCH_SIZE_kB_median": f_kb, "WRITE_SIZE_kB_median": w_kb,
               "hbm_bytes_per_launch": (2 * f_kb + w_kb) * 1024.0,
               "correction": "FETCH_SIZE x2 (gfx950 16-B/lane reads), WRITE_SIZE x1; kB = 1024 B",
               "workload": f"tools/rowpass_workload.py 40 {H} {mb}"}
        with open(os.path.join(prof, f"{tag}_rowpass{sfx}_pmc.json"), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res))
    mfma = os.path.join(d, "pmc_mfma" + sfx, "run_counter_collection.csv")
    if os.path.exists(mfma):
        # SQ_VALU_MFMA_BUSY_CYCLES sums each MFMA's busy cycles on its SIMD over the
        # chip; GRBM_GUI_ACTIVE sums the busy cycles of the 8 XCDs (MI355X_MICROARCH.md),
        # so one XCD's span is /8
        busy, nb = pmc_per_dispatch(mfma, "rowpass_kernel", "SQ_VALU_MFMA_BUSY_CYCLES")
        grbm, ng = pmc_per_dispatch(mfma, "rowpass_kernel", "GRBM_GUI_ACTIVE")
        sqb, ns = pmc_per_dispatch(mfma, "rowpass_kernel", "SQ_BUSY_CYCLES")
        n_f32, n_bf16 = rowpass_mfma_counts(H, mb)
        busy_expected = 32 * n_f32 + 16 * n_bf16
        res = {"kernel": kernel, "hidden": H, "minibatch": mb, "dispatches": [nb, ng, ns],
               "SQ_VALU_MFMA_BUSY_CYCLES_median": busy, "GRBM_GUI_ACTIVE_median": grbm,
               "SQ_BUSY_CYCLES_median": sqb,
               "xcd_cycles": grbm / 8.0 if grbm else None,
               "mfma_busy_frac": busy / (grbm / 8.0 * 1024) if busy and grbm else None,
               "mfma_instructions_per_launch": n_f32 + n_bf16,
               "mfma_f32_16x16x4_per_launch": n_f32, "mfma_bf16_16x16x32_per_launch": n_bf16,
               "busy_cycles_expected": busy_expected,
               "busy_over_expected": busy / busy_expected if busy else None,
               "definition": MFMA_DEF, "workload": f"tools/rowpass_workload.py 40 {H} {mb}"}
        with open(os.path.join(prof, f"{tag}_rowpass{sfx}_mfma_pmc.json"), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res))


def policy_summary(d, tag, prof, sfx, H, n):
    """The rollout's policy kernel (both agents' forward, n rows each; 32-row
    workgroups).  H 256: 8 waves, each 2 row tiles x 2 column tiles: fc1 (K
    padded to 32) 32 f32 per wave, fc2 as split-bf16 8 chunks x 4 tiles x 6 =
    192 per wave.  H 64: 4 waves, one column tile each: fc1 16, fc2 2 chunks x
    16 = 48 f32 per wave."""
    pol = os.path.join(d, "pmc_policy_mfma" + sfx, "run_counter_collection.csv")
    if not os.path.exists(pol):
        return
    busy, nb = pmc_per_dispatch(pol, "policy_kernel", "SQ_VALU_MFMA_BUSY_CYCLES")
    grbm, ng = pmc_per_dispatch(pol, "policy_kernel", "GRBM_GUI_ACTIVE")
    wgs = 2 * (n // 32)
    n_f32, n_bf16 = (wgs * 8 * 32, wgs * 8 * 192) if H == 256 else (wgs * 4 * 48, 0)
    busy_expected = 32 * n_f32 + 16 * n_bf16
    nw = 8 if H == 256 else H // 16
    res = {"kernel": f"policy_kernel<{H}, {nw}, 0>", "hidden": H, "num_envs": n, "agents": 2,
           "dispatches": [nb, ng], "SQ_VALU_MFMA_BUSY_CYCLES_median": busy, "GRBM_GUI_ACTIVE_median": grbm,
           "xcd_cycles": grbm / 8.0 if grbm else None,
           "mfma_busy_frac": busy / (grbm / 8.0 * 1024) if busy and grbm else None,
           "mfma_instructions_per_launch": n_f32 + n_bf16, "busy_cycles_expected": busy_expected,
           "busy_over_expected": busy / busy_expected if busy else None,
           "definition": MFMA_DEF, "workload": f"tools/policy_workload.py 40 {H} {n}"}
    with open(os.path.join(prof, f"{tag}_policy{sfx}_mfma_pmc.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


def env_extra(d, tag, prof):
    """The env kernel's in-rollout kernel stats, its mid-episode durations per
    env count (kernel trace split by grid size), and its FP64 VALU work."""
    hbm_peak, bytes_per_env = 8000.0, 381
    ks = os.path.join(d, "env_rollout", "run_kernel_stats.csv")
    if os.path.exists(ks):
        rows = kernel_stats(ks, os.path.join(prof, f"{tag}_env_rollout_kernel_stats.csv"))
        env = [r for r in rows if "step_kernel_wide" in r["Name"]]
        pol = [r for r in rows if "policy_kernel" in r["Name"]]
        if env:
            us = float(env[0]["AverageNs"]) / 1e3
            res = {"kernel": env[0]["Name"], "calls": int(env[0]["Calls"]), "avg_launch_us": us, "num_envs": 16384,
                   "achieved_GBs": 16384 * bytes_per_env / (us * 1e-6) / 1e9,
                   "hbm_frac": 16384 * bytes_per_env / (us * 1e-6) / 1e9 / hbm_peak,
                   "env_steps_per_s": 16384 / (us * 1e-6),
                   "policy_kernel_avg_us": float(pol[0]["AverageNs"]) / 1e3 if pol else None,
                   "workload": "tools/env_workload.py rollout 1: VecTrainer.collect() x 2 (16384 envs, H 256, "
                               "2048 steps, hipGraph chunks); every env-step dispatch is an in-rollout launch",
                   "bytes_per_env_step": bytes_per_env}
            with open(os.path.join(prof, f"{tag}_env_rollout.json"), "w") as f:
                json.dump(res, f, indent=1)
            print(json.dumps(res))
    tr = os.path.join(d, "env_sweep", "run_kernel_trace.csv")
    if os.path.exists(tr):
        by = {}
        for r in csv.DictReader(open(tr)):
            if "step_kernel_wide" not in r["Kernel_Name"]:
                continue
            gk = [k for k in r if k.startswith("Grid_Size")]
            grid = 1
            for k in gk:
                grid *= max(1, int(float(r[k])))
            by.setdefault(grid, []).append((int(r["Dispatch_Id"]),
                                            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
        res = {"workload": "tools/env_workload.py sweep 200: per env count 256 warm-up steps (U(-1.6,1.6) actions), "
                           "then 200 mid-episode launches; kernel trace, the last 200 dispatches per grid size",
               "bytes_per_env_step": bytes_per_env, "sizes": {}}
        # grid = threads = 4 waves x 64 lanes per 64 envs -> envs = grid / 4
        for grid, v in sorted(by.items()):
            v.sort()
            us = sorted(t for _, t in v[-200:])
            n = grid // 4
            avg = sum(us) / len(us)
            res["sizes"][str(n)] = {"dispatches": len(us), "avg_launch_us": avg, "median_launch_us": us[len(us) // 2],
                                    "env_steps_per_s": n / (avg * 1e-6),
                                    "hbm_frac": n * bytes_per_env / (avg * 1e-6) / 1e9 / hbm_peak}
        with open(os.path.join(prof, f"{tag}_env_sweep.json"), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res))
    fp = os.path.join(d, "pmc_env_fp64", "run_counter_collection.csv")
    if os.path.exists(fp):
        names = sorted({r["Counter_Name"] for r in csv.DictReader(open(fp))})
        vals = {c: pmc_per_dispatch(fp, "step_kernel", c, last=40)[0] for c in names}
        flops = 0.0
        for c, v in vals.items():
            if v is None or not c.endswith("F64"):
                continue
            w = 2 if "FMA" in c else (0 if "MFMA" in c else 1)
            flops += 64.0 * w * v
        sweep = os.path.join(prof, f"{tag}_env_sweep.json")
        us = None
        if os.path.exists(sweep):
            us = json.load(open(sweep))["sizes"].get("16384", {}).get("avg_launch_us")
        res = {"kernel": "satenv step_kernel_wide<true, 64>, 16384 envs mid-episode", "counters_per_launch": vals,
               "fp64_flops_per_launch": flops,
               "avg_launch_us": us, "fp64_tflops_achieved": flops / (us * 1e-6) / 1e12 if us else None,
               "fp64_vector_peak_tflops": 78.6,
               "fp64_frac": flops / (us * 1e-6) / 1e12 / 78.6 if us else None,
               "definition": "FLOPs = 64 lanes x (ADD + MUL + TRANS + 2 x FMA) F64 wave instructions, the last 40 "
                             "dispatches (median); duration = the sweep trace's 16384-env average (the same "
                             "workload, unprofiled); peak = AMD's FP64 vector figure (not in the local guide)",
               "workload": "tools/env_workload.py 40"}
        with open(os.path.join(prof, f"{tag}_env_fp64_pmc.json"), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res))


if __name__ == "__main__":
    main()
