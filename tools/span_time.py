#!/usr/bin/env python3
"""Development tool (not shipped, not a test): the in-graph minibatch step
time (event-timed graph replays of the update, 16-minibatch groups) and each
kernel's live launch span (satrl_span_probe: max wave exit - min wave start)
inside those graphs, for the library SATRL_LIB_PATH selects (default: the
product build).  Optional: the rollout's policy and env-step spans.
Usage: python tools/span_time.py H mb[,mb...] [reps] [rollout]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
from satrl.ppo import FusedMinibatch, PPOLearner  # noqa: E402
from satrl.spans import SpanProbe  # noqa: E402
from satrl.trainer import args_param  # noqa: E402

tag = os.path.basename(os.environ.get("SATRL_LIB_PATH", "product"))


def step_and_spans(H, mb, n=20):
    B = 16 * mb
    a = args_param(hidden_width=H, mini_batch_size=mb, batch_size=B, chkpt_dir="/tmp")
    L = PPOLearner(a, "pursuer", graph_group=16)
    g = torch.Generator(device="cuda").manual_seed(0)
    src = torch.randn((B, 32), device="cuda", generator=g)
    src[:, 21:24] = -1.0 - torch.rand((B, 3), device="cuda", generator=g)
    perm = torch.randperm(B, device="cuda", generator=g)
    L.sync_w2t()
    st = FusedMinibatch(L, mb, 16)
    for _ in range(3):
        st.run(src, perm)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        st.run(src, perm)
    e1.record()
    torch.cuda.synchronize()
    step = e0.elapsed_time(e1) * 1e3 / (n * 16)
    with SpanProbe(64 << 20) as pr:
        sp = FusedMinibatch(L, mb, 16)
        for _ in range(3):
            sp.run(src, perm)
        torch.cuda.synchronize()
    return step, pr.summary(), pr.gaps(["rowpass", "dw2", "reduce", "adam"])


def rollout_spans(H, n_envs=16384, n=64):
    from satrl.trainer import VecTrainer
    a = args_param(batch_size=n_envs * 64, mini_batch_size=4096, hidden_width=H, K_epochs=1, max_episode_steps=1000,
                   num_envs=n_envs, horizon=64, seed=0, chkpt_dir="/tmp")
    tr = VecTrainer(a, flag=0, d_capture=15000.0)
    tr.collect()
    tr.collect()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    tr.collect()
    e1.record()
    torch.cuda.synchronize()
    step = e0.elapsed_time(e1) * 1e3 / 64
    tr._graphs.clear()
    with SpanProbe(256 << 20) as pr:
        tr.collect()                          # captures the chunk graph with the probe on, replays it
        tr.collect()
        torch.cuda.synchronize()
    return step, pr.summary()


if __name__ == "__main__":
    H = int(sys.argv[1])
    mbs = [int(x) for x in sys.argv[2].split(",")]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    for _ in range(reps):
        for mb in mbs:
            step, s, gp = step_and_spans(H, mb)
            ks = " ".join(f"{k} {v['median_us']:.2f}" for k, v in s.items())
            gs = " ".join(f"{k} {v['median_us']:.2f}" for k, v in gp.items())
            print(f"[{tag}] H {H} mb {mb:5d}: step {step:6.2f} us | span medians: {ks} | gaps: {gs}", flush=True)
    if len(sys.argv) > 4 and sys.argv[4] == "rollout":
        step, s = rollout_spans(H)
        ks = " ".join(f"{k} {v['median_us']:.2f}" for k, v in s.items())
        print(f"[{tag}] H {H} rollout 16384 envs: step {step:6.2f} us | span medians: {ks}", flush=True)
