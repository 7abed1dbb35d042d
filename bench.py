#!/usr/bin/env python3
"""Benchmark: one "step" = one PPO iteration of the hot path on N GPUs:
a rollout of T=2048 env-steps for each of 16384 envs per GPU (actor forward
x2 agents -> HIP Gaussian sampling -> HIP FP64 env step, hipGraph chunks),
critic values, HIP GAE scan, global advantage normalisation, and the PPO
update (K=10 epochs x minibatch 4096, hidden 256, Adam, grad clip).
Workload = BASELINE.json configs[2]; scaling is weak (16384 envs per GPU).

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Rank 0 prints ONE JSON line.  value = all env-steps processed by all ranks
(N_total * T * K) / max-over-ranks wall time of the K timed iterations.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))

METRIC = "env-steps/sec + PPO updates/sec at N_envs=16384, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_MFMA_PEAK_TFS = 157.3     # MI355X_MICROARCH.md: FP32 matrix 157.3 TF spec
BF16_MFMA_PEAK_TFS = 2500.0    # MI355X_MICROARCH.md: dense BF16 matrix ~2.5 PF
SURROGATE_FLOP_PER_ENV = 2 * (5 * 256 + 256 * 128 + 128 * 64 + 64 * 10)   # ImprovedNN forward, algorithmic
ENV_BYTES_PER_STEP = 381       # DESIGN.md "Roofline": state 16 f64 + 3 i32 planes r/w, actions, obs, reward, done


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--num-envs", type=int, default=16384, help="envs per GPU")
    ap.add_argument("--horizon", type=int, default=2048)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--minibatch", type=int, default=4096)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--d-capture", type=float, default=15000.0)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=6.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-iters", type=int, default=200)
    ap.add_argument("--graph-group", type=int, default=64, help="minibatches per replayed update hipGraph")
    ap.add_argument("--force-dist", action="store_true",
                    help="init the nccl process group even at world size 1 (rehearses the DP update path)")
    ap.add_argument("--surrogate", action="store_true",
                    help="config 5: ImprovedNN surrogate (bf16) evaluated on every env step of the rollout")
    return ap.parse_args()


def cpu_baseline(seconds, n, T, H, mb, epochs):
    """The same PPO iteration on host cores, from bounded samples of each
    part, scaled to one iteration (N envs x T steps, K epochs of mb-row
    minibatches) -> whole-iteration env-steps/s, the unit of ``value``:
      env step   oracle/satenv_oracle.c (the C restatement), n envs from the
                 reference reset state with autoreset (Flag 0, U(-1.6,1.6)
                 f32 actions), chunks of 64 steps until ~`seconds`, OpenMP
                 over envs;
      policy     both agents' choose_action on n states and the critic values
                 (oracle/ppo_cpu.py, torch-CPU f32 as ppo_continuous.py);
      GAE        the reference's python reverse loop (oracle.gae_flat) on 2
                 envs x T, scaled to n envs and divided by the thread count
                 (envs are independent: perfect parallel assumed);
      update     oracle/ppo_cpu.py minibatch steps (mb rows, H hidden),
                 x (n*T/mb)*epochs."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import ppo_cpu
    threads = max(1, min(16, os.cpu_count() or 1))
    chunk = 64
    rng = np.random.default_rng(0)
    pa = rng.uniform(-1.6, 1.6, (chunk, n, 3)).astype(np.float32)
    ea = rng.uniform(-1.6, 1.6, (chunk, n, 3)).astype(np.float32)
    ro = O.Rollout(n, d_capture=15000.0, max_episode_steps=1000)
    steps, dt = 0, 0.0
    while dt < seconds and steps < 256 * chunk:
        t0 = time.perf_counter()
        ro.run(pa, ea, nthreads=threads)
        dt += time.perf_counter() - t0
        steps += chunk
    t_env = dt / steps
    t_pol, t_val, t_mb = ppo_cpu.time_learning_side(n, H, mb, threads)
    g = np.random.default_rng(1)
    r = g.standard_normal(T).astype(np.float32)
    vs = g.standard_normal(T).astype(np.float32)
    dn = (g.random(T) < 0.01).astype(np.float32)
    t0 = time.perf_counter()
    for _ in range(2):
        O.gae_flat(r, vs, vs, dn, dn)
    t_gae_env = (time.perf_counter() - t0) / 2
    t_iter = (T * (t_env + t_pol) + (T + 1) * t_val + n * t_gae_env / threads
              + epochs * (n * T // mb) * t_mb)
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": n * T / t_iter, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"one PPO iteration ({n} envs x {T} steps, H {H}, {epochs} epochs x mb {mb}) on "
                      f"{threads} threads of '{model}' (os.cpu_count()={os.cpu_count()}), scaled from samples: "
                      f"env step = oracle C restatement, {n} envs x {steps} steps with autoreset (Flag 0, "
                      f"U(-1.6,1.6) actions, d_capture 15000, max_episode_steps 1000); policy/values/update = "
                      f"oracle/ppo_cpu.py torch-CPU f32 (8 policy steps, 2 value passes, 24 minibatches); GAE = "
                      f"the reference's python loop on 2 envs x {T}",
            "iteration_s": t_iter,
            "env_step_only_env_steps_per_s": n / t_env,
            "s_per_env_step_batch": t_env, "s_per_policy_step_both_agents": t_pol,
            "s_per_value_pass": t_val, "s_per_update_minibatch": t_mb, "s_gae_per_env_python": t_gae_env,
            "seconds": dt}


def rd_cpu_baseline():
    """One reference-default reachable-domain grid (RD_single_pulse.py params
    :9-20) on the C restatement and its Curve_fitting on the numpy/scipy
    restatement, 1 core: (ms per grid, ms per Curve_fitting)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import ellipse_oracle as EO
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        mx, mn = O.reachable_domain(1e7, 0.2, np.pi / 2, 500.0, 1, 200, 200)
    t1 = time.perf_counter()
    for _ in range(reps):
        EO.curve_fitting(mx, mn)
    t2 = time.perf_counter()
    return (t1 - t0) / reps * 1e3, (t2 - t1) / reps * 1e3


def workload_name(a, world):
    """Which BASELINE.json config this run is (configs[1..3]), or a plain description."""
    desc = (f"num_envs={a.num_envs}/GPU x {world} GPU, hidden={a.hidden}, horizon={a.horizon}, GAE lambda=0.95, "
            f"minibatch={a.minibatch}, {a.epochs} PPO epochs")
    if a.surrogate:
        desc += ", ImprovedNN surrogate bf16 per env-step"
    if a.horizon == 2048 and a.minibatch == 4096 and a.epochs == 10:
        if world == 1 and a.num_envs == 16384 and a.hidden == 256 and a.surrogate:
            return "BASELINE.json configs[4]: " + desc
        if world == 1 and a.num_envs == 16384 and a.hidden == 256:
            return "BASELINE.json configs[2]: " + desc
        if world == 1 and a.num_envs == 4096 and a.hidden == 64:
            return "BASELINE.json configs[1]: " + desc
        if world == 8 and a.num_envs == 8192:
            return "BASELINE.json configs[3]: " + desc
    return desc


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    pg = None
    if world > 1 or a.force_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        pg = dist.group.WORLD

    from satrl.trainer import VecTrainer, args_param
    args = args_param(batch_size=a.num_envs * a.horizon, mini_batch_size=a.minibatch, hidden_width=a.hidden,
                      K_epochs=a.epochs, max_episode_steps=1000, num_envs=a.num_envs, horizon=a.horizon, seed=0,
                      max_train_steps=int(3e6), chkpt_dir="/tmp", surrogate=a.surrogate,
                      update_graph_group=a.graph_group)
    tr = VecTrainer(args, flag=0, d_capture=a.d_capture, pg=pg, env_offset=rank * a.num_envs)

    def barrier():
        if pg is not None:
            dist.barrier()

    timers = {}
    for _ in range(a.warmup):
        tr.iteration()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        stats = tr.iteration(timers)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if pg is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    n_total = a.num_envs * world
    env_steps = n_total * a.horizon * a.steps
    value = env_steps / elapsed

    # ---- roofline of the dominant kernel (satrl_ppo_rowpass, ~60% of the update):
    # HIP events around back-to-back launches on the stream it is launched on
    # (torch's current stream, see satrl._lib.stream_ptr), same inputs as the update.
    L = tr.learner
    st = L.stepper(a.minibatch)
    src = tr.buf.packed
    g = torch.Generator(device="cuda").manual_seed(1)
    idx = torch.randperm(src.shape[0], device="cuda", generator=g)[:a.minibatch].contiguous()
    for _ in range(10):
        st.rowpass(src, idx)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.kernel_iters):
        st.rowpass(src, idx)
    e1.record()
    torch.cuda.synchronize()
    rowpass_us = e0.elapsed_time(e1) * 1e3 / a.kernel_iters
    rowpass_flop = st.rowpass_flops(a.hidden, a.minibatch)
    rowpass_tfs = rowpass_flop / (rowpass_us * 1e-6) / 1e12
    # the same kernel's average inside the update's graphs (after each step's
    # Adam rewrote W2/W2T, so the weights come from MALL, not a warm L2), from
    # the committed rocprofv3 kernel stats of this command
    in_update_us = None
    ks_file = os.path.join(ROOT, "profiles", "r1_bench_kernel_stats.csv")
    if os.path.exists(ks_file):
        import csv
        with open(ks_file) as f:
            for r in csv.DictReader(f):
                if "rowpass_kernel<%d" % a.hidden in r["name"].replace(" ", ""):
                    in_update_us = float(r["avg_ns"]) / 1e3
    traffic = None
    pmc_file = os.path.join(ROOT, "profiles", "r1_rowpass_pmc.json")
    if os.path.exists(pmc_file):
        with open(pmc_file) as f:
            pmc = json.load(f)
        if pmc.get("hidden") == a.hidden and pmc.get("minibatch") == a.minibatch:
            traffic = pmc["hbm_bytes_per_launch"]

    # ---- env kernel (FP64 step, autoreset): HIP events around eager launches on its stream
    env = tr.env
    pa = tr.buf.act[0].clone()
    ea = torch.empty_like(pa).uniform_(-1.6, 1.6)
    obs = torch.empty((a.num_envs, 18), dtype=torch.float32, device="cuda")
    rew = torch.empty(a.num_envs, dtype=torch.float32, device="cuda")
    dn = torch.empty(a.num_envs, dtype=torch.uint8, device="cuda")
    for _ in range(10):
        env.step_autoreset(pa, ea, obs, rew, dn)
    e0.record()
    for _ in range(a.kernel_iters):
        env.step_autoreset(pa, ea, obs, rew, dn)
    e1.record()
    torch.cuda.synchronize()
    env_us = e0.elapsed_time(e1) * 1e3 / a.kernel_iters
    env_gbs = a.num_envs * ENV_BYTES_PER_STEP / (env_us * 1e-6) / 1e9
    env_traffic = None
    pmc_file = os.path.join(ROOT, "profiles", "r1_env_pmc.json")
    if os.path.exists(pmc_file):
        with open(pmc_file) as f:
            pmc = json.load(f)
        if pmc.get("num_envs") == a.num_envs:
            env_traffic = pmc["hbm_bytes_per_launch"]

    # ---- north-star sweep: the env kernel alone at num_envs 4k / 16k / 64k on this GPU
    # (autoreset, U(-1.6,1.6) f32 actions cycled from 64 pre-drawn sets, 256 untimed
    # steps first so episodes are mid-flight and the danger-zone solves are in their
    # steady mix, then kernel_iters timed launches)
    from satrl.env import VecSatellites
    env_sweep = {}
    gs = torch.Generator(device="cuda").manual_seed(7)
    for n_sw in (4096, 16384, 65536):
        e_sw = VecSatellites(n_sw, d_capture=a.d_capture, max_episode_steps=1000)
        e_sw.reset(0)
        acts = (torch.rand((64, 2, n_sw, 3), device="cuda", generator=gs) * 3.2 - 1.6).contiguous()
        o_sw = torch.empty((n_sw, 18), dtype=torch.float32, device="cuda")
        r_sw = torch.empty(n_sw, dtype=torch.float32, device="cuda")
        d_sw = torch.empty(n_sw, dtype=torch.uint8, device="cuda")
        for k in range(256):
            e_sw.step_autoreset(acts[k % 64, 0], acts[k % 64, 1], o_sw, r_sw, d_sw)
        e0.record()
        for k in range(a.kernel_iters):
            e_sw.step_autoreset(acts[k % 64, 0], acts[k % 64, 1], o_sw, r_sw, d_sw)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.kernel_iters
        gbs = n_sw * ENV_BYTES_PER_STEP / (us * 1e-6) / 1e9
        env_sweep[str(n_sw)] = {"avg_launch_us": us, "env_steps_per_s": n_sw / (us * 1e-6), "achieved_GBs": gbs,
                                "hbm_frac": gbs / HBM_PEAK_GBS}
        del e_sw, acts

    # ---- north-star sweep, end to end: the rollout (both agents' policy kernel ->
    # Philox sampling -> env step, hipGraph chunks) at num_envs 4k / 16k / 64k, a
    # 256-step horizon after one untimed collect (graphs captured, episodes mid-flight)
    rollout_sweep = {}
    for n_sw in (4096, 16384, 65536):
        a_sw = args_param(batch_size=n_sw * 256, mini_batch_size=a.minibatch, hidden_width=a.hidden, K_epochs=1,
                          max_episode_steps=1000, num_envs=n_sw, horizon=256, seed=0, max_train_steps=int(3e6),
                          chkpt_dir="/tmp")
        tr_sw = VecTrainer(a_sw, flag=0, d_capture=a.d_capture)
        tr_sw.collect()
        torch.cuda.synchronize()
        e0.record()
        tr_sw.collect()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        rollout_sweep[str(n_sw)] = {"ms_per_256_steps": ms, "env_steps_per_s": n_sw * 256 / (ms * 1e-3)}
        del tr_sw

    # ---- §8f propagators: RK4 two-body + J2 batch kernel, and the env step in RK4-CW mode
    from satrl.env import rk4_j2
    g = torch.Generator(device="cuda").manual_seed(3)
    rv = torch.empty((a.num_envs, 6), dtype=torch.float64, device="cuda")
    rv[:, :3] = torch.randn((a.num_envs, 3), dtype=torch.float64, device="cuda", generator=g) * 7000.0
    rv[:, 3:] = torch.randn((a.num_envs, 3), dtype=torch.float64, device="cuda", generator=g) * 5.0
    rk_steps = 100
    rk4_j2(rv, 1.0, 2)
    e0.record()
    rk4_j2(rv, 1.0, rk_steps)
    e1.record()
    torch.cuda.synchronize()
    rk4_ms = e0.elapsed_time(e1)
    env_rk = VecSatellites(a.num_envs, d_capture=a.d_capture, max_episode_steps=1000, propagator=1, rk4_substeps=10)
    env_rk.reset(0)
    for _ in range(10):
        env_rk.step_autoreset(pa, ea, obs, rew, dn)
    e0.record()
    for _ in range(a.kernel_iters):
        env_rk.step_autoreset(pa, ea, obs, rew, dn)
    e1.record()
    torch.cuda.synchronize()
    env_rk_us = e0.elapsed_time(e1) * 1e3 / a.kernel_iters

    # ---- §8f rank 4: reachable-domain grid (RD_single_pulse.py:40-148), the reference's
    # default 1 x 201 x 201 direction grid for a batch of orbits in one launch
    from satrl import reachable as RD
    rd_sets = 256
    gr = np.random.default_rng(5)
    rd_orb = RD.orbits_tensor(gr.uniform(7e6, 5e7, rd_sets), gr.uniform(0.0, 0.8, rd_sets),
                              gr.uniform(0.05, 2 * np.pi - 0.05, rd_sets), gr.uniform(50.0, 1000.0, rd_sets),
                              device="cuda")
    rd_out = RD.reachable_domain_grid(rd_orb, 1, 200, 200)
    rd_reach = int((rd_out[2] == 1).sum())
    rd_iters = 5
    e0.record()
    for _ in range(rd_iters):
        RD.reachable_domain_grid(rd_orb, 1, 200, 200)
    e1.record()
    torch.cuda.synchronize()
    rd_ms = e0.elapsed_time(e1) / rd_iters
    ell, ell_info = RD.ellipse_fit(*rd_out)
    e0.record()
    for _ in range(rd_iters):
        RD.ellipse_fit(*rd_out)
    e1.record()
    torch.cuda.synchronize()
    ell_ms = e0.elapsed_time(e1) / rd_iters
    ell_ok = int((ell_info > 0).sum())
    del rd_out, ell, ell_info

    # ---- config 5 kernel: ImprovedNN surrogate (bf16 MFMA) on every env's current orbit
    from satrl.surrogate import Surrogate
    sur = tr.surrogate if tr.surrogate is not None else Surrogate(device="cuda", seed=0)
    sur_out = torch.empty((a.num_envs, 10), dtype=torch.float32, device="cuda")
    for _ in range(10):
        sur.env_forward(env, out=sur_out)
    e0.record()
    for _ in range(a.kernel_iters):
        sur.env_forward(env, out=sur_out)
    e1.record()
    torch.cuda.synchronize()
    sur_us = e0.elapsed_time(e1) * 1e3 / a.kernel_iters
    sur_flop = a.num_envs * SURROGATE_FLOP_PER_ENV
    sur_tfs = sur_flop / (sur_us * 1e-6) / 1e12

    rollout_ms = sum(timers["rollout_ms"]) / len(timers["rollout_ms"])
    update_ms = sum(timers["update_ms"]) / len(timers["update_ms"])
    gae_ms = sum(timers["gae_ms"]) / len(timers["gae_ms"])
    H = a.hidden
    flop_per_transition_epoch = 6 * (18 * H + H * H + 3 * H) + 6 * (18 * H + H * H + H)
    upd_flops = a.num_envs * a.horizon * a.epochs * flop_per_transition_epoch
    upd_tfs = upd_flops / (update_ms * 1e-3) / 1e12
    n_minibatches = a.epochs * ((a.num_envs * a.horizon) // a.minibatch)

    if rank == 0:
        host_baseline = not a.no_cpu_baseline and world == 1          # rank 0 at N = 1 only
        cpu = cpu_baseline(a.cpu_baseline_seconds, a.num_envs, a.horizon, a.hidden, a.minibatch,
                           a.epochs) if host_baseline else None
        rd_cpu_ms = rd_cpu_baseline() if host_baseline else None
        out = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64+f32",
            "data": "synthetic: reference reset state, random-init (orthogonal, seed 0) policies",
            "config": {"workload": workload_name(a, world),
                       "num_envs_per_gpu": a.num_envs, "num_envs_total": n_total, "horizon": a.horizon,
                       "hidden": a.hidden, "minibatch_per_gpu": a.minibatch, "epochs": a.epochs,
                       "d_capture": a.d_capture, "parallelism": f"dp{world}"},
            "ppo_updates_per_s": a.steps / elapsed,
            "rollout_env_steps_per_s": n_total * a.horizon / (rollout_ms * 1e-3),
            "rollout_sweep_num_envs": rollout_sweep,
            "rollout_ms": rollout_ms, "gae_ms": gae_ms, "update_ms": update_ms,
            "env_kernel_env_steps_per_s": a.num_envs / (env_us * 1e-6),
            "minibatch_steps_per_s": n_minibatches / (update_ms * 1e-3),
            "episodes_finished_total": float(stats[0]),
            "roofline": {"kernel": f"satrl_ppo_rowpass<{a.hidden},{a.hidden // 16}> (hand-written HIP, f32 MFMA 16x16x4)",
                         "bound": "mfma",
                         "achieved": rowpass_tfs, "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": rowpass_tfs / FP32_MFMA_PEAK_TFS, "traffic": traffic,
                         "avg_launch_us": rowpass_us, "flop_per_launch": rowpass_flop,
                         "in_update_avg_launch_us": in_update_us,
                         "in_update_frac": (rowpass_flop / (in_update_us * 1e-6) / 1e12 / FP32_MFMA_PEAK_TFS
                                            if in_update_us else None),
                         "in_update_source": "profiles/r1_bench_kernel_stats.csv (rocprofv3 average over all "
                                             "rowpass launches of this command, nearly all inside the update)",
                         "traffic_source": "profiles/r1_rowpass_pmc.json (FETCH_SIZE x2 + WRITE_SIZE, bytes/launch)",
                         "note": "f32 MFMA; one net per workgroup of 32 rows, each streams that net's fc2 weights "
                                 "from L2 per phase (DESIGN.md 3.4)"},
            "roofline_env": {"kernel": "satenv step_kernel<autoreset> (hand-written HIP, FP64)", "bound": "hbm",
                             "achieved": env_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": env_gbs / HBM_PEAK_GBS,
                             "avg_launch_us": env_us, "bytes_per_env_step": ENV_BYTES_PER_STEP,
                             "traffic": env_traffic,
                             "traffic_source": "profiles/r1_env_pmc.json (FETCH_SIZE x2 + WRITE_SIZE, bytes/launch, "
                                               "16384 envs mid-episode)",
                             "note": "algorithmic bytes; the kernel is FP64 latency bound (DESIGN.md)",
                             "sweep_num_envs": env_sweep},
            "roofline_update": {"bound": "mfma", "achieved": upd_tfs, "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                                "frac": upd_tfs / FP32_MFMA_PEAK_TFS,
                                "flop_per_transition_epoch": flop_per_transition_epoch},
            "propagators": {"rk4_j2_state_steps_per_s": a.num_envs * rk_steps / (rk4_ms * 1e-3),
                            "rk4_j2_sample": f"{a.num_envs} states x {rk_steps} RK4 steps (h=1 s), one launch",
                            "env_rk4_cw_avg_launch_us": env_rk_us,
                            "env_rk4_cw_env_steps_per_s": a.num_envs / (env_rk_us * 1e-6)},
            "surrogate": {"kernel": "satenv_surrogate (ImprovedNN 5-256-128-64-10, bf16 MFMA 16x16x32, f32 acc)",
                          "in_rollout": bool(a.surrogate), "avg_launch_us": sur_us,
                          "env_steps_per_s": a.num_envs / (sur_us * 1e-6), "bound": "mfma",
                          "achieved": sur_tfs, "peak": BF16_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                          "frac": sur_tfs / BF16_MFMA_PEAK_TFS, "flop_per_env": SURROGATE_FLOP_PER_ENV,
                          "note": "latency bound: 91 KB of packed weights staged into LDS per workgroup; "
                                  "FP64 orbital elements per env"},
            "reachable_domain": {"grids_per_s": rd_sets / (rd_ms * 1e-3), "ms_per_launch": rd_ms,
                                 "sample": f"{rd_sets} random orbits x 201 x 201 directions (RD_single_pulse "
                                           "defaults N1=1, N2=N3=200), one launch incl. output zero-fill",
                                 "reachable_directions": rd_reach,
                                 "cpu_oracle_ms_per_grid": rd_cpu_ms[0] if rd_cpu_ms else None,
                                 "ellipse_fit_ms_per_launch": ell_ms,
                                 "ellipse_fits_per_s": 2 * rd_sets / (ell_ms * 1e-3), "ellipse_fits_ok": ell_ok,
                                 "grid_plus_fit_orbits_per_s": rd_sets / ((rd_ms + ell_ms) * 1e-3),
                                 "cpu_oracle_ms_per_curve_fitting": rd_cpu_ms[1] if rd_cpu_ms else None},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if pg is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
