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


def dw2_kernel_name(st):
    """Which hand-written kernel computes dW2 on a FusedMinibatch's path."""
    if st.kx(st.mb):
        return "dw2_kx (split-bf16 from k-packed planes)"
    return "rowpass_dw2 (fused)" if st.fused_dw2 else "dw2_kernel (f32)"


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
    ap.add_argument("--dp-minibatch", choices=("auto", "global", "per_gpu"), default="auto",
                    help="data parallelism: 'global' = --minibatch is the global minibatch, each of N ranks steps "
                         "minibatch/N of its rows per Adam step (the reference's semantics, SURVEY 8e); 'per_gpu' = "
                         "every rank steps --minibatch rows (global minibatch N x --minibatch); 'auto' (default) = "
                         "global for BASELINE configs[3] (65536 envs over 8 GPUs) and at N = 1, per_gpu for the "
                         "weak-scaling series of configs[2] (16384 envs per GPU at N = 2/4/8)")
    ap.add_argument("--allreduce", choices=("rccl", "peer"), default="rccl",
                    help="N > 1: the update's per-minibatch gradient all-reduce: RCCL (ncclAllReduce + reduce_dp in "
                         "the graphs) or the peer kernel (satrl_ppo_allreduce_peer: two-shot over IPC-mapped "
                         "buffers, fused with reduce_dp); the line times the other one beside it")
    ap.add_argument("--profile-tag", default="r6", help="profiles/<tag>_* files the rocprof cross-check fields read")
    ap.add_argument("--global-slice", type=int, default=256,
                    help="N > 1: minibatches of the configs[3]-semantics slice timed after the run (global "
                         "minibatch --minibatch, i.e. --minibatch/N rows per rank per Adam step); 0 = off")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: rehearse the launch, barrier, max-over-ranks timing and the rank-0 JSON line "
                         "with gloo all-reduces of the gradient bucket's size (CPU test of the N-rank path)")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank on cuda:0 over gloo (RCCL refuses two ranks on "
                         "one GPU); use a small --num-envs/--horizon, the update is eager there")
    return ap.parse_args()


def host_cores():
    """Cores this process may use on the host: its CPU affinity, capped by a
    cgroup CPU quota and by OMP_NUM_THREADS when set (the GPU box gives a
    one-GPU job a 16-core share of a larger host).  Returns (cores, how)."""
    n = len(os.sched_getaffinity(0))
    how = [f"affinity {n}"]
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(float(q) / float(per))))
            how.append(f"cgroup quota {q}/{per}")
    except (OSError, ValueError):
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        n = min(n, int(os.environ["OMP_NUM_THREADS"]))
        how.append(f"OMP_NUM_THREADS {os.environ['OMP_NUM_THREADS']}")
    return max(1, n), ", ".join(how)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def host_env_rate(n, steps, threads, seed=0):
    """env-steps/s of the product's host build (satenv_cpu_step_autoreset,
    OpenMP over envs) from reset, U(-1.6, 1.6) f32 actions, Flag 0,
    d_capture 15000, max_episode_steps 1000."""
    import torch
    from satrl.env import VecSatellites
    env = VecSatellites(n, device="cpu", d_capture=15000.0, max_episode_steps=1000, threads=threads)
    env.reset(0)
    g = np.random.default_rng(seed)
    acts = torch.from_numpy(g.uniform(-1.6, 1.6, (min(steps, 64), 2, n, 3)).astype(np.float32))
    obs = torch.empty((n, 18), dtype=torch.float32)
    rew = torch.empty(n, dtype=torch.float32)
    dn = torch.empty(n, dtype=torch.uint8)
    t0 = time.perf_counter()
    for k in range(steps):
        env.step_autoreset(acts[k % len(acts), 0], acts[k % len(acts), 1], obs, rew, dn)
    return n * steps / (time.perf_counter() - t0)


def cpu_baseline(seconds, n, T, H, mb, epochs):
    """The same PPO iteration on host cores, scaled from bounded samples of
    each part to one iteration (N envs x T steps, K epochs of mb-row
    minibatches) -> whole-iteration env-steps/s, the unit of ``value``:
      env step   the product's host build (satenv_cpu_*: the kernels' FP64
                 step source through g++, bit-identical to the glibc
                 reference and to oracle/satenv_oracle.c), n envs from reset
                 with autoreset, U(-1.6,1.6) f32 actions, OpenMP over envs,
                 chunks of 64 steps until ~`seconds`;
      policy     both agents' choose_action on n states and the critic values
                 (oracle/ppo_cpu.py, torch-CPU f32 as ppo_continuous.py);
      GAE        the reference's python reverse loop (oracle.gae_flat) on 2
                 envs x T, scaled to n envs and divided by the thread count;
      update     oracle/ppo_cpu.py minibatch steps (mb rows, H hidden),
                 x (n*T/mb)*epochs.
    Threads: the host cores this job may use (host_cores()).  Plus the
    SURVEY 8(d) env-only leg: 4096 envs x 100 steps on 1 thread and on all
    of them."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import ppo_cpu
    threads, how = host_cores()
    steps, t_env = 0, 0.0
    chunk = 64
    while t_env < seconds and steps < 256 * chunk:
        rate = host_env_rate(n, chunk, threads, seed=steps)
        t_env += n * chunk / rate
        steps += chunk
    t_env_step = t_env / steps
    env_only_1 = host_env_rate(4096, 100, 1)
    env_only_all = host_env_rate(4096, 100, threads)
    t_pol, t_val, t_mb = ppo_cpu.time_learning_side(n, H, mb, threads)
    g = np.random.default_rng(1)
    r = g.standard_normal(T).astype(np.float32)
    vs = g.standard_normal(T).astype(np.float32)
    dn = (g.random(T) < 0.01).astype(np.float32)
    t_gae_env = float("inf")
    for _ in range(2):                         # the faster of two samples (shared host)
        t0 = time.perf_counter()
        O.gae_flat(r, vs, vs, dn, dn)
        t_gae_env = min(t_gae_env, time.perf_counter() - t0)
    t_iter = (T * (t_env_step + t_pol) + (T + 1) * t_val + n * t_gae_env / threads
              + epochs * (n * T // mb) * t_mb)
    total = os.cpu_count() or threads
    return {"value": n * T / t_iter, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "host_threads_total": total, "cores_how": how,
            "sample": f"one PPO iteration ({n} envs x {T} steps, H {H}, {epochs} epochs x mb {mb}) on {threads} "
                      f"threads of '{cpu_model()}' ({how}; the host has {total} hardware threads), scaled from "
                      f"samples: env step = the product's host build satenv_cpu_step_autoreset, {n} envs x {steps} "
                      f"steps from reset (Flag 0, U(-1.6,1.6) actions, d_capture 15000, max_episode_steps 1000); "
                      f"policy/values/update = oracle/ppo_cpu.py torch-CPU f32 (fastest of 3 samples of 2 policy "
                      f"steps, of 2 value passes, of 3 samples of 8 minibatches); GAE = the reference's python "
                      f"loop on 1 env x {T}, faster of 2",
            "iteration_s": t_iter,
            "env_step_only_env_steps_per_s": n / t_env_step,
            "env_only_4096x100": {"threads_1": env_only_1, f"threads_{threads}": env_only_all,
                                  "per_core": env_only_all / threads,
                                  "all_host_threads_linear_extrapolation": env_only_all / threads * total},
            "s_per_env_step_batch": t_env_step, "s_per_policy_step_both_agents": t_pol,
            "s_per_value_pass": t_val, "s_per_update_minibatch": t_mb, "s_gae_per_env_python": t_gae_env,
            "seconds": t_env}


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
    """Which BASELINE.json config this run is (configs[1..4]), or a plain description."""
    gmb = a.minibatch if (world == 1 or a.dp_minibatch == "global") else a.minibatch * world
    desc = (f"num_envs={a.num_envs}/GPU x {world} GPU, hidden={a.hidden}, horizon={a.horizon}, GAE lambda=0.95, "
            f"global minibatch={gmb} ({gmb // world if world > 1 else gmb} rows per GPU per Adam step), "
            f"{a.epochs} PPO epochs")
    if a.surrogate:
        desc += ", ImprovedNN surrogate bf16 per env-step (trained on the reference's golden pairs)"
    if a.horizon == 2048 and gmb == 4096 and a.epochs == 10:
        if world == 1 and a.num_envs == 16384 and a.hidden == 256 and a.surrogate:
            return "BASELINE.json configs[4]: " + desc
        if world == 1 and a.num_envs == 16384 and a.hidden == 256:
            return "BASELINE.json configs[2]: " + desc
        if world == 1 and a.num_envs == 4096 and a.hidden == 64:
            return "BASELINE.json configs[1]: " + desc
        if world == 8 and a.num_envs == 8192 and a.hidden == 256:
            return "BASELINE.json configs[3]: " + desc
    if (world > 1 and a.dp_minibatch == "per_gpu" and a.num_envs == 16384 and a.hidden == 256
            and a.horizon == 2048 and a.minibatch == 4096 and a.epochs == 10 and not a.surrogate):
        return ("weak-scaling series of BASELINE.json configs[2] (each GPU runs configs[2] on its env shard, "
                "gradients averaged per minibatch): " + desc)
    return desc


def dp_mode(a, world):
    """--dp-minibatch auto: the reference's global minibatch wherever the total
    env count is a configuration's own (N = 1, configs[3]); per_gpu for the
    weak-scaling series, where the global minibatch would multiply the number
    of sequential Adam steps by N and the per-GPU work would not stay fixed."""
    if a.dp_minibatch != "auto":
        return a.dp_minibatch
    return "global" if world == 1 or (world == 8 and a.num_envs == 8192) else "per_gpu"


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher: start N fresh copies of this
    command, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous
    on 127.0.0.1), and wait for them.  The parent never imports torch or
    touches a GPU (a process that has initialised the GPU must not exec).
    Rank 0 prints the JSON line.  If a rank fails, the others are stopped and
    the parent exits with the failing rank's code."""
    import signal
    import subprocess
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
    signal.signal(signal.SIGTERM, lambda *_: (stop(), sys.exit(143)))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                sys.stderr.write(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the others\n")
                stop()
        time.sleep(0.05)
    return rc


def main():
    a = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus))
    world = int(world_env or "1")
    if world != a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}: one rank per GPU, the two must agree")
    if a.dry_run:
        sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
        from satrl import dist as _dist
        return _dist.run_or_exit(dry_run, a, world, world=world)
    sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
    from satrl import dist as _dist
    return _dist.run_or_exit(run, a, world, world=world)


def dry_run(a, world):
    """The N-rank launch / barrier / max-over-ranks timing / rank-0 report
    path without a GPU: gloo process group, each "step" one all-reduce of the
    per-minibatch gradient bucket (142 860 f32 at H 256)."""
    import datetime
    import torch
    import torch.distributed as dist
    from satrl import dist as _dist
    rank = int(os.environ.get("RANK", "0"))
    pg = None
    if world > 1:
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=_dist.dp_timeout_s()))
        pg = dist.group.WORLD
        assert dist.get_world_size() == a.gpus, (dist.get_world_size(), a.gpus)
    g = torch.ones(142860, dtype=torch.float32)
    cnt = torch.ones(1, dtype=torch.float32)
    _dist.sum_inplace_(cnt, pg)
    for _ in range(a.warmup):
        _dist.sum_inplace_(g, pg)
    if pg is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        _dist.sum_inplace_(g, pg)
    if os.environ.get("SATRL_DRY_RUN_FAIL_RANK") == str(rank):     # failure-path test hook
        os._exit(7)
    if pg is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64)
    if pg is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    n_gpus = dist.get_world_size() if pg is not None else 1
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "env-steps/s", "n_gpus": n_gpus,
                          "steps": a.steps, "warmup": a.warmup, "ms_per_step": float(t.item()) / a.steps * 1e3,
                          "dry_run": True, "ranks_seen": int(cnt.item()),
                          "config": {"workload": workload_name(a, n_gpus), "parallelism": f"dp{n_gpus}"}}),
              flush=True)
    if pg is not None:
        dist.destroy_process_group()


def run(a, world):
    import datetime
    import torch
    import torch.distributed as dist
    from satrl import dist as _dist

    a.dp_minibatch = dp_mode(a, world)
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if a.one_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    pg = None
    if world > 1 or a.force_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        timeout = datetime.timedelta(seconds=_dist.dp_timeout_s())
        if a.one_device:
            dist.init_process_group("gloo", timeout=timeout)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
        pg = dist.group.WORLD
        if dist.get_world_size() != a.gpus:
            raise RuntimeError(f"process group has {dist.get_world_size()} ranks, --gpus {a.gpus}")
    n_gpus = dist.get_world_size() if pg is not None else 1

    from satrl.trainer import VecTrainer, args_param
    args = args_param(batch_size=a.num_envs * a.horizon, mini_batch_size=a.minibatch, hidden_width=a.hidden,
                      K_epochs=a.epochs, max_episode_steps=1000, num_envs=a.num_envs, horizon=a.horizon, seed=0,
                      max_train_steps=int(3e6), chkpt_dir="/tmp", surrogate=a.surrogate,
                      update_graph_group=a.graph_group, dp_minibatch=a.dp_minibatch,
                      allreduce=a.allreduce if pg is not None else "rccl")
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

    n_total = a.num_envs * n_gpus
    env_steps = n_total * a.horizon * a.steps
    value = env_steps / elapsed

    # ---- roofline of the dominant kernel (satrl_ppo_rowpass, ~55% of the update).
    # Live, in the update's own conditions: eager minibatch steps (rowpass ->
    # dW2 -> reduce -> Adam, each step's Adam rewriting the weights the next
    # rowpass streams) with HIP events recorded on the launch stream around
    # every rowpass; a GPU-side spin queued first lets the host enqueue the
    # whole run ahead of the GPU, so the kernels run back to back as in the
    # update's graphs.  (This continues training; it is after the timed region.)
    L = tr.learner
    mb_local = tr.mb_local
    st = L.stepper(mb_local)
    src = tr.buf.packed
    g = torch.Generator(device="cuda").manual_seed(1)
    stage = src[torch.randperm(src.shape[0], device="cuda", generator=g)[:mb_local]].contiguous()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    spin = torch.empty(1 << 28, dtype=torch.float32, device="cuda")   # fallback backlog: 1 GiB of fills
    try:
        e0.record()
        torch.cuda._sleep(10 ** 7)
        e1.record()
        torch.cuda.synchronize()
        sleep_cycles_per_ms = 10 ** 7 / e0.elapsed_time(e1)
    except (RuntimeError, AttributeError):
        sleep_cycles_per_ms = None

    def backlog(ms):
        if sleep_cycles_per_ms:
            torch.cuda._sleep(int(ms * sleep_cycles_per_ms))
        else:
            for _ in range(int(ms / 0.2) + 1):
                spin.fill_(1.0)

    def timed_pairs(n, fn, ahead_ms):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for k in range(10):
            fn(k, None)
        torch.cuda.synchronize()
        backlog(ahead_ms)
        for k in range(n):
            fn(k, evs[k])
        torch.cuda.synchronize()
        ts = sorted(x.elapsed_time(y) * 1e3 for x, y in evs)
        return sum(ts) / n, ts[n // 2]

    def timed_run(n, fn, ahead_ms):
        """Average time per call of n back-to-back calls (one event pair over the run)."""
        for k in range(10):
            fn(k)
        torch.cuda.synchronize()
        backlog(ahead_ms)
        e0.record()
        for k in range(n):
            fn(k)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / n

    # marginal cost of the rowpass on the minibatch chain (whole chain minus the
    # chain without the rowpass), the headline; plus per-launch event brackets
    # (each event marker adds its own fence to the stream, so they read high)
    t_chain = timed_run(a.kernel_iters, lambda k: st.step(stage, None), 60.0)
    t_rest = timed_run(a.kernel_iters, lambda k: st.step(stage, None, skip_rowpass=True), 40.0)
    rowpass_us = t_chain - t_rest
    rowpass_ev_us, rowpass_med = timed_pairs(a.kernel_iters, lambda k, ev: st.step(stage, None, events=ev), 60.0)
    rowpass_flop = st.step_kernel_flops(mb_local)        # + the fused dW2 product at H = 64
    rowpass_tfs = rowpass_flop / (rowpass_us * 1e-6) / 1e12
    # warm-L2 figure: back-to-back rowpass launches alone (W2/W2T stay in L2)
    rp_launch = st.rowpass_dw2 if st.fused_dw2 else (st.rowpass_kx if st.kx(mb_local) else st.rowpass)
    for _ in range(10):
        rp_launch(stage, None)
    e0.record()
    for _ in range(a.kernel_iters):
        rp_launch(stage, None)
    e1.record()
    torch.cuda.synchronize()
    b2b_us = e0.elapsed_time(e1) * 1e3 / a.kernel_iters
    # rocprof cross-checks from the committed profiles of this command / the PMC workloads
    # the committed kernel stats profile the default command (1 GPU, 16384 envs,
    # H 256, mb 4096; profiles/<tag>_bench_kernel_stats.csv) and configs[1] (4096
    # envs, H 64, mb 4096; ..._bench_configs1_kernel_stats.csv): other shapes time
    # other launches, so they fall back to the live figures
    profiled_shape = world == 1 and a.num_envs == 16384 and a.hidden == 256 and mb_local == 4096
    ks_suffix = {(1, 16384, 256, 4096): "", (1, 4096, 64, 4096): "_configs1"}.get(
        (world, a.num_envs, a.hidden, mb_local))
    ks_file = (os.path.join(ROOT, "profiles", f"{a.profile_tag}_bench{ks_suffix}_kernel_stats.csv")
               if ks_suffix is not None else None)

    def prof_avg_us(kname):
        if ks_file is None or not os.path.exists(ks_file):
            return None
        import csv
        with open(ks_file) as f:
            for r in csv.DictReader(f):
                if kname in r["name"].replace(" ", ""):
                    return float(r["avg_ns"]) / 1e3
        return None

    # PMC summaries per shape: the bench's H 256 ones, "_h64" for configs[1]'s
    # (tools/profile_round.sh), each used only when its shape is this run's
    sfx = {256: "", 64: "_h64"}.get(a.hidden, "_none")

    def pmc(kind, **match):
        pmc_file = os.path.join(ROOT, "profiles", f"{a.profile_tag}_{kind}{sfx}_pmc.json")
        if os.path.exists(pmc_file):
            with open(pmc_file) as f:
                d = json.load(f)
            if all(d.get(k) == v for k, v in match.items()):
                return d["hbm_bytes_per_launch"]
        return None

    rowpass_prof_us = prof_avg_us("rowpass_kernel<%d" % a.hidden)

    # ---- live launch spans (satrl_span_probe, satrl/spans.py): every kernel's
    # duration measured in THIS run, inside the update's own hipGraphs -- a fresh
    # stepper captured while the probe is on runs two graph groups of minibatch
    # steps (its kernels' SPAN instantiations add one 16-B store per wave at its
    # exit) -- and over eager rollout steps queued behind a GPU spin.  These are
    # the headline durations; the committed rocprof averages stay beside them.
    from satrl.ppo import FusedMinibatch
    from satrl.spans import SpanProbe
    upd_spans, roll_spans = {}, {}
    perm_sp = torch.randperm(src.shape[0], device="cuda", generator=g)[:2 * L.graph_group * mb_local].contiguous()
    with SpanProbe() as probe:
        stp = FusedMinibatch(L, mb_local, L.graph_group, use_graph=True)
        stp.run(src, perm_sp)                    # capture (each node keeps its record region), then two replays
        torch.cuda.synchronize()
    upd_spans = probe.summary()
    upd_gaps = probe.gaps(["rowpass", "dw2", "reduce", "adam"])
    del stp
    # the rollout: one whole training rollout (T steps, both agents' policy kernel
    # and the env step per step) through freshly captured chunk graphs, so every
    # env-step launch of the rollout has its span (the trainer's graphs are kept
    # aside and put back afterwards)
    saved_graphs = tr._graphs
    tr._graphs = {}
    with SpanProbe(int(2.2 * a.horizon * (2 * a.num_envs // 32 * 8 + a.num_envs // 64 * 4) * 16) + (64 << 20)) as probe:
        e0.record()
        tr.collect()
        e1.record()
        torch.cuda.synchronize()
    roll_spans = probe.summary()
    roll_span_run_ms = e0.elapsed_time(e1)
    tr._graphs = saved_graphs
    rowpass_live_us = upd_spans.get("rowpass", {}).get("avg_us")
    head_us = rowpass_live_us if rowpass_live_us else rowpass_us
    traffic = pmc("rowpass", hidden=a.hidden, minibatch=mb_local)
    # the rollout's policy kernel (both agents' forward, the (num_envs x hidden)
    # GEMMs): per row and agent fc1 2*18*H + H, fc2 2*H*H + H, mean layer 2*3*H + 3
    policy_roof = None
    pol_nw = 8 if a.hidden == 256 else a.hidden // 16      # waves per policy workgroup (csrc kPolNW at H 256)
    pol_prof_us = prof_avg_us("policy_kernel<%d;%d;0>" % (a.hidden, pol_nw))
    pol_us = roll_spans.get("policy_act", {}).get("avg_us") or pol_prof_us
    if pol_us:
        pol_flop = 2 * a.num_envs * (2 * 18 * a.hidden + a.hidden + 2 * a.hidden * a.hidden + a.hidden
                                     + 2 * 3 * a.hidden + 3)
        pol_tfs = pol_flop / (pol_us * 1e-6) / 1e12
        policy_roof = {"kernel": f"policy_kernel<{a.hidden},{pol_nw},0> (both agents' choose_action; "
                                 + ("fc1 on f32 MFMA, fc2 on split-bf16 MFMA, FLOPs counted as f32)" if a.hidden == 256
                                    else "f32 MFMA)"),
                       "bound": "mfma", "achieved": pol_tfs, "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                       "frac": pol_tfs / FP32_MFMA_PEAK_TFS, "avg_launch_us": pol_us, "flop_per_launch": pol_flop,
                       "timing": ("live launch span in this run (satrl_span_probe: max wave exit - min wave start, "
                                  "s_memrealtime) averaged over every launch of one whole training rollout"
                                  if roll_spans.get("policy_act") else "rocprofv3 average (committed profile)"),
                       "rocprof_avg_launch_us": pol_prof_us,
                       "rocprof_source": (f"profiles/{os.path.basename(ks_file)} (committed profile of this command)"
                                          if ks_file else None)}
        pol_file = os.path.join(ROOT, "profiles", f"{a.profile_tag}_policy{sfx}_mfma_pmc.json")
        d = None
        if os.path.exists(pol_file):
            with open(pol_file) as f:
                d = json.load(f)
        # (only a pass over this very kernel and shape: hidden width and env count)
        if d is not None and d.get("hidden") == a.hidden and d.get("num_envs") == a.num_envs:
            policy_roof["mfma_utilisation"] = {
                "mfma_busy_cycles_per_launch": d["SQ_VALU_MFMA_BUSY_CYCLES_median"],
                "mfma_busy_frac_dispatch_window": d["mfma_busy_frac"],
                "source": f"profiles/{a.profile_tag}_policy{sfx}_mfma_pmc.json (lower bound: the --pmc dispatch "
                          "window includes the profiler's set-up)"}
    mfma_util = None                   # SQ_VALU_MFMA_BUSY_CYCLES pass (tools/profile_round.sh)
    mfma_file = os.path.join(ROOT, "profiles", f"{a.profile_tag}_rowpass{sfx}_mfma_pmc.json")
    if os.path.exists(mfma_file):
        with open(mfma_file) as f:
            d = json.load(f)
        if d.get("hidden") == a.hidden and d.get("minibatch") == mb_local:
            mfma_util = {"mfma_busy_cycles_per_launch": d["SQ_VALU_MFMA_BUSY_CYCLES_median"],
                         "mfma_busy_frac_dispatch_window": d["mfma_busy_frac"],
                         "source": f"profiles/{a.profile_tag}_rowpass{sfx}_mfma_pmc.json (lower bound: the --pmc "
                                   "dispatch window includes the profiler's set-up)"}

    # ---- env kernel: in the rollout (live: eager rollout steps -- policy kernel,
    # then the env step between HIP events -- after the timed region, the
    # trainer's own envs and policy), and mid-episode under uniform actions
    # (the sweep below)
    t_roll = [0]

    def roll_step(k, ev):
        tr._policy_step(t_roll[0] % a.horizon, events=ev)
        t_roll[0] += 1

    def roll_policy_only(k):
        tr._policy_step(t_roll[0] % a.horizon, env=False)
        t_roll[0] += 1

    env_us = (timed_run(a.kernel_iters, lambda k: roll_step(k, None), 40.0)
              - timed_run(a.kernel_iters, roll_policy_only, 30.0))
    env_ev_us, env_med = timed_pairs(a.kernel_iters, roll_step, 40.0)
    env_live_gbs = a.num_envs * ENV_BYTES_PER_STEP / (env_us * 1e-6) / 1e9
    # rocprof figures from the env-only profile passes (tools/profile_round.sh): the
    # in-rollout average (a process running nothing but the training rollout) and the
    # mid-episode averages per env count (kernel trace split by grid size)
    env_roll_prof, env_sweep_prof = None, None
    if profiled_shape:
        f_roll = os.path.join(ROOT, "profiles", f"{a.profile_tag}_env_rollout.json")
        f_sweep = os.path.join(ROOT, "profiles", f"{a.profile_tag}_env_sweep.json")
        if os.path.exists(f_roll):
            env_roll_prof = json.load(open(f_roll))
        if os.path.exists(f_sweep):
            env_sweep_prof = json.load(open(f_sweep))["sizes"]
    env_prof_us = env_roll_prof["avg_launch_us"] if env_roll_prof else None
    env_fp64 = None
    f_fp64 = os.path.join(ROOT, "profiles", f"{a.profile_tag}_env_fp64_pmc.json")
    if os.path.exists(f_fp64):
        d = json.load(open(f_fp64))
        env_fp64 = {"fp64_flops_per_launch": d["fp64_flops_per_launch"], "fp64_frac": d["fp64_frac"],
                    "peak_tflops": d["fp64_vector_peak_tflops"],
                    "source": f"profiles/{a.profile_tag}_env_fp64_pmc.json (16384 envs mid-episode)"}
    env_span_us = roll_spans.get("env_step", {}).get("avg_us")
    env_head_us = env_span_us if env_span_us else env_us
    env_gbs = a.num_envs * ENV_BYTES_PER_STEP / (env_head_us * 1e-6) / 1e9
    env_traffic = pmc("env", num_envs=a.num_envs)
    env = tr.env
    pa = tr.buf.act[0].clone()
    ea = torch.empty_like(pa).uniform_(-1.6, 1.6)
    obs = torch.empty((a.num_envs, 18), dtype=torch.float32, device="cuda")
    rew = torch.empty(a.num_envs, dtype=torch.float32, device="cuda")
    dn = torch.empty(a.num_envs, dtype=torch.uint8, device="cuda")

    # ---- single-GPU figures (sweeps, propagators, RD grid, surrogate): measured at N = 1;
    # at N > 1 every rank would repeat them on its own GPU, so the N-rank run skips them
    env_sweep, rollout_sweep = None, None
    if world == 1:
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
        # propagator 2: solve_ivp RK45 on the CW orbit_ode (satellite_function.py:783-839)
        env_rk.set_params(propagator=2)
        env_rk.reset(0)
        for _ in range(10):
            env_rk.step_autoreset(pa, ea, obs, rew, dn)
        e0.record()
        for _ in range(a.kernel_iters):
            env_rk.step_autoreset(pa, ea, obs, rew, dn)
        e1.record()
        torch.cuda.synchronize()
        env_rk45_us = e0.elapsed_time(e1) * 1e3 / a.kernel_iters
        del env_rk

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

    # ---- data parallelism (N > 1): the per-minibatch gradient all-reduce alone, and a
    # bounded slice of the configs[3] semantics (global minibatch --minibatch over the N
    # ranks: minibatch/N rows per rank per Adam step, the all-reduce on the chain)
    dp_out = {}
    if pg is not None:
        dp = {"world": n_gpus, "backend": dist.get_backend(pg), "dp_minibatch": tr.dp_minibatch,
              "allreduce": a.allreduce,
              "gradient_bucket_bytes": L.G.numel() * 4, "minibatch_step_us": t_chain,
              "dw2_kernel": dw2_kernel_name(st)}
        if L.comm is not None:
            scratch = torch.zeros_like(L.G)
            L.comm.warm(scratch)
            barrier()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.kernel_iters):
                L.comm.all_reduce_sum_(scratch)
            e1.record()
            torch.cuda.synchronize()
            ar = torch.tensor([e0.elapsed_time(e1) * 1e3 / a.kernel_iters], dtype=torch.float64, device="cuda")
            dist.all_reduce(ar, op=dist.ReduceOp.MAX)
            dp["allreduce_us"] = float(ar.item())
            dp["allreduce_timing"] = ("HIP events on the compute stream around kernel_iters back-to-back "
                                      "ncclAllReduce calls (satrl.rccl, the call the update's graphs capture), "
                                      "max over ranks")
        # the peer all-reduce (fused with reduce_dp) on the same bucket, A/B beside RCCL
        try:
            from satrl.peer import PeerComm
            peer = L.peer if L.peer is not None else PeerComm(pg, L.G.numel(), "cuda", L.H)
            scratch = torch.randn(L.G.numel(), device="cuda")
            nsq_s = torch.zeros_like(st.nsq[0])
            steps_s = torch.zeros(2, dtype=torch.float64, device="cuda")
            for _ in range(5):
                peer.all_reduce_dp_(a.hidden, mb_local, scratch, nsq_s, steps_s)
            barrier()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.kernel_iters):
                peer.all_reduce_dp_(a.hidden, mb_local, scratch, nsq_s, steps_s)
            e1.record()
            torch.cuda.synchronize()
            pr = torch.tensor([e0.elapsed_time(e1) * 1e3 / a.kernel_iters], dtype=torch.float64, device="cuda")
            perr = torch.tensor([float(peer.error())], dtype=torch.float64, device="cuda")
            dist.all_reduce(pr, op=dist.ReduceOp.MAX)
            dist.all_reduce(perr, op=dist.ReduceOp.MAX)
            dp["peer_allreduce_us"] = float(pr.item())
            dp["peer_allreduce_error"] = bool(perr.item())
            dp["peer_allreduce_timing"] = ("HIP events around kernel_iters back-to-back satrl_ppo_allreduce_peer "
                                           "calls (the all-reduce of the gradient bucket fused with reduce_dp: "
                                           "its norms and step counters), max over ranks")
            if peer is not L.peer:
                peer.close()
        except Exception as exc:                       # noqa: BLE001 -- reported, not fatal to the line
            dp["peer_allreduce_error"] = f"{type(exc).__name__}: {exc}"[:300]
        if a.global_slice > 0 and tr.dp_minibatch == "per_gpu" and a.minibatch % n_gpus == 0:
            mbg = a.minibatch // n_gpus
            stg = L.stepper(mbg)
            gperm = torch.randperm(src.shape[0], device="cuda", generator=g)[:a.global_slice * mbg].contiguous()
            stg.run(src, gperm)                      # plans, captures the graphs, warms
            torch.cuda.synchronize()
            barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            stg.run(src, gperm)
            torch.cuda.synchronize()
            barrier()
            torch.cuda.synchronize()
            tg = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device="cuda")
            dist.all_reduce(tg, op=dist.ReduceOp.MAX)
            us_g = float(tg.item()) / a.global_slice * 1e6
            steps_c3 = a.epochs * (65536 * a.horizon) // a.minibatch
            dp["configs3_semantics_slice"] = {
                "global_minibatch": a.minibatch, "rows_per_rank": mbg, "minibatches": a.global_slice,
                "us_per_global_minibatch_step": us_g,
                "dw2_kernel": dw2_kernel_name(stg),
                "note": ("global-minibatch mode (the reference's BatchSampler(..., 4096) semantics, "
                         "ppo_continuous.py:215) timed on a bounded slice after the run: wall time of "
                         f"{a.global_slice} minibatch steps between barriers, max over ranks; the "
                         "all-reduce is on every step's critical path"),
                "configs3_update_s_projected": steps_c3 * us_g * 1e-6,
                "configs3_projection": f"BASELINE configs[3] (65536 envs, T {a.horizon}, {a.epochs} epochs, global "
                                       f"minibatch {a.minibatch}) has {steps_c3} global minibatch steps per update"}
        dp_out = {"data_parallel": dp}

    rollout_ms = sum(timers["rollout_ms"]) / len(timers["rollout_ms"])
    update_ms = sum(timers["update_ms"]) / len(timers["update_ms"])
    gae_ms = sum(timers["gae_ms"]) / len(timers["gae_ms"])
    H = a.hidden
    flop_per_transition_epoch = 6 * (18 * H + H * H + 3 * H) + 6 * (18 * H + H * H + H)
    upd_flops = a.num_envs * a.horizon * a.epochs * flop_per_transition_epoch
    upd_tfs = upd_flops / (update_ms * 1e-3) / 1e12
    n_minibatches = a.epochs * ((a.num_envs * a.horizon) // tr.mb_local)

    # self-consistency: the kernels of one step, by their live spans, cannot
    # take longer than the step itself on the timed region's clock
    def span_check(kinds, spans, live_us, what):
        got = [spans[k]["avg_us"] for k in kinds if k in spans]
        tot = sum(got) if len(got) == len(kinds) else None
        ok = tot is not None and tot <= live_us
        if not ok:
            print(f"bench: {what}: kernel spans {tot} us exceed the live step {live_us:.2f} us", file=sys.stderr)
        return {"kernels": kinds, "sum_of_span_avgs_us": tot, "live_step_us": live_us, "pass": ok,
                "rule": f"sum of the kernels' live span averages <= the timed region's {what} time per step"}
    upd_kinds = ["rowpass", "reduce", "adam"] + ([] if st.fused_dw2 else ["dw2"])
    upd_check = span_check(upd_kinds, upd_spans, update_ms * 1e3 / n_minibatches, "update (minibatch step)")
    roll_check = span_check(["policy_act", "env_step"], roll_spans, rollout_ms * 1e3 / a.horizon, "rollout step")

    if rank == 0:
        host_baseline = not a.no_cpu_baseline and world == 1          # rank 0 at N = 1 only
        cpu = cpu_baseline(a.cpu_baseline_seconds, a.num_envs, a.horizon, a.hidden, a.minibatch,
                           a.epochs) if host_baseline else None
        rd_cpu_ms = rd_cpu_baseline() if host_baseline else None
        out = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": n_gpus, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64+f32",
            "data": "synthetic: reference reset state, random-init (orthogonal, seed 0) policies",
            "config": {"workload": workload_name(a, n_gpus),
                       "num_envs_per_gpu": a.num_envs, "num_envs_total": n_total, "horizon": a.horizon,
                       "hidden": a.hidden, "minibatch_global": tr.global_minibatch,
                       "minibatch_rows_per_gpu": tr.mb_local, "dp_minibatch": tr.dp_minibatch,
                       "minibatch_sampler": tr.sampler, "epochs": a.epochs,
                       "d_capture": a.d_capture, "parallelism": f"dp{n_gpus}"},
            "ppo_updates_per_s": a.steps / elapsed,
            "rollout_env_steps_per_s": n_total * a.horizon / (rollout_ms * 1e-3),
            "rollout_sweep_num_envs": rollout_sweep,
            "rollout_ms": rollout_ms, "gae_ms": gae_ms, "update_ms": update_ms,
            "env_kernel_env_steps_per_s": a.num_envs / (env_us * 1e-6),
            "minibatch_steps_per_s": n_minibatches / (update_ms * 1e-3),
            "episodes_finished_total": float(stats[0]),
            "roofline": {"kernel": (f"satrl_ppo_rowpass_dw2<{a.hidden},{a.hidden // 16}> (hand-written HIP, f32 MFMA "
                                    "16x16x4; the dW2 product fused in)" if st.fused_dw2 else
                                    f"satrl_ppo_rowpass{'_kx' if st.kx(mb_local) else ''}<{a.hidden},{a.hidden // 16}> "
                                    "(hand-written HIP; fc1 / [dW1|db1] on f32 MFMA 16x16x4, the two HxH products on "
                                    "split-bf16 v_mfma_f32_16x16x32_bf16, FLOPs counted as f32)"
                                    if a.hidden == 256 else
                                    f"satrl_ppo_rowpass<{a.hidden},{a.hidden // 16}> (hand-written HIP, f32 MFMA 16x16x4)"),
                         "bound": "mfma",
                         "achieved": rowpass_flop / (head_us * 1e-6) / 1e12, "peak": FP32_MFMA_PEAK_TFS,
                         "unit": "TFLOP/s",
                         "frac": rowpass_flop / (head_us * 1e-6) / 1e12 / FP32_MFMA_PEAK_TFS, "traffic": traffic,
                         "avg_launch_us": head_us, "flop_per_launch": rowpass_flop, "rows_per_launch": mb_local,
                         "timing": ("live in-update kernel duration measured in this run: the launch span "
                                    "(satrl_span_probe: max wave exit - min wave start, s_memrealtime, 100 MHz) "
                                    "averaged over every rowpass launch of two replays of the update's own 64-"
                                    "minibatch hipGraph; the committed rocprof average and the live marginal beside it"
                                    if rowpass_live_us else
                                    "live marginal cost (the span probe gave no rowpass launches)"),
                         "live_span_avg_launch_us": rowpass_live_us,
                         "update_kernel_spans": upd_spans,
                         "update_boundary_gaps": upd_gaps,
                         "update_boundary_gaps_timing": ("next launch's first wave start minus the previous launch's "
                                                         "last wave exit (span clock), one replay of the update's "
                                                         "64-minibatch graph"),
                         "live_marginal_avg_launch_us": rowpass_us,
                         "live_marginal_frac": rowpass_tfs / FP32_MFMA_PEAK_TFS,
                         "live_marginal_timing": "HIP events on the launch stream: kernel_iters minibatch steps "
                                                 "(rowpass -> dW2 -> reduce -> Adam, each Adam rewriting the weights "
                                                 "the next rowpass streams, as in the update) minus the same steps "
                                                 "without the rowpass, per launch, behind a GPU spin; it carries the "
                                                 "launch boundary the rowpass adds to the chain",
                         "minibatch_step_us": t_chain,
                         "event_bracketed_avg_launch_us": rowpass_ev_us, "event_bracketed_median_us": rowpass_med,
                         "rocprof_avg_launch_us": rowpass_prof_us,
                         "rocprof_frac": (rowpass_flop / (rowpass_prof_us * 1e-6) / 1e12 / FP32_MFMA_PEAK_TFS
                                          if rowpass_prof_us else None),
                         "rocprof_source": (f"profiles/{os.path.basename(ks_file)} (COMMITTED rocprofv3 profile of this "
                                            "command, not this run: average over all rowpass launches, nearly all in "
                                            "the update's graphs)" if ks_file else None),
                         "check": upd_check,
                         "back_to_back_avg_launch_us": b2b_us,
                         "back_to_back_frac": rowpass_flop / (b2b_us * 1e-6) / 1e12 / FP32_MFMA_PEAK_TFS,
                         "traffic_source": f"profiles/{a.profile_tag}_rowpass{sfx}_pmc.json (FETCH_SIZE x2 + WRITE_SIZE, "
                                           "bytes/launch)",
                         "mfma_utilisation": mfma_util,
                         "note": "f32 MFMA; one net per workgroup of 32 rows, each streams that net's fc2 weights "
                                 "from L2 per phase (DESIGN.md 3.4)"},
            "roofline_env": {"kernel": "satenv step_kernel_wide<autoreset, 64> (hand-written HIP, FP64)", "bound": "hbm",
                             "achieved": env_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": env_gbs / HBM_PEAK_GBS,
                             "avg_launch_us": env_head_us, "bytes_per_env_step": ENV_BYTES_PER_STEP,
                             "num_envs": a.num_envs,
                             "timing": ("live in-rollout kernel duration measured in this run: the launch span "
                                        "(satrl_span_probe) averaged over every env-step launch of one whole "
                                        "training rollout (T steps through freshly captured chunk graphs, after the "
                                        "timed region); the committed rocprof average beside it"
                                        if env_span_us else "live marginal cost (no span)"),
                             "span_rollout_ms": roll_span_run_ms,
                             "live_span_avg_launch_us": env_span_us,
                             "rollout_kernel_spans": roll_spans,
                             "check": roll_check,
                             "live_marginal_avg_launch_us": env_us, "live_marginal_GBs": env_live_gbs,
                             "live_marginal_timing": "HIP events: kernel_iters eager rollout steps (policy kernel -> "
                                                     "env step) on the trainer's envs after the timed region, minus "
                                                     "the same steps without the env step, per launch",
                             "event_bracketed_avg_launch_us": env_ev_us, "event_bracketed_median_us": env_med,
                             "rocprof_avg_launch_us": env_prof_us,
                             "rocprof_source": (f"profiles/{a.profile_tag}_env_rollout.json / _env_rollout_kernel_stats"
                                                ".csv (COMMITTED profile, not this run)"),
                             "rocprof_mid_episode_by_num_envs": env_sweep_prof,
                             "fp64_utilisation": env_fp64,
                             "traffic": env_traffic,
                             "traffic_source": f"profiles/{a.profile_tag}_env_pmc.json (FETCH_SIZE x2 + WRITE_SIZE, "
                                               "bytes/launch, 16384 envs mid-episode, uniform actions)",
                             "note": "algorithmic bytes; the kernel is FP64 latency bound (DESIGN.md)",
                             "sweep_mid_episode_uniform_actions": env_sweep},
            "roofline_update": {"bound": "mfma", "achieved": upd_tfs, "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                                "frac": upd_tfs / FP32_MFMA_PEAK_TFS,
                                "flop_per_transition_epoch": flop_per_transition_epoch},
            "roofline_policy": policy_roof,
            "cpu_baseline": cpu,
        }
        if world == 1:
            out.update({
                "propagators": {"rk4_j2_state_steps_per_s": a.num_envs * rk_steps / (rk4_ms * 1e-3),
                                "rk4_j2_sample": f"{a.num_envs} states x {rk_steps} RK4 steps (h=1 s), one launch",
                                "env_rk4_cw_avg_launch_us": env_rk_us,
                                "env_rk4_cw_env_steps_per_s": a.num_envs / (env_rk_us * 1e-6),
                                "env_rk45_cw_avg_launch_us": env_rk45_us,
                                "env_rk45_cw_env_steps_per_s": a.num_envs / (env_rk45_us * 1e-6),
                                "note": "rk4_cw: propagator 1 (RK4, 10 substeps); rk45_cw: propagator 2, the "
                                        "reference's solve_ivp RK45 on orbit_ode (satellite_function.py:783-839); "
                                        "RK4 stage weights: launch-uniform, held in scalar registers (an LDS table "
                                        "would hold the same doubles and add a load per use)"},
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
                                     "cpu_oracle_ms_per_curve_fitting": rd_cpu_ms[1] if rd_cpu_ms else None}})
        out.update(dp_out)
        print(json.dumps(out), flush=True)
    if pg is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
