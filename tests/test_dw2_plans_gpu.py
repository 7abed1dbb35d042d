"""Reproducible dW2 (the hipBLASLt fc2-weight-gradient GEMM at H = 256,
csrc/dw2_blas.cpp): the solution of every shape is pinned from the committed
table (satrl/dw2_plans.json), under data parallelism to rank 0's, so every
process and rank sums its split-K partial tiles the same way
(ppo_continuous.py:226-238 is one process; VERDICT r2 "dW2 plans can differ
across processes").  Plus the split-chain mode's per-chain workspaces."""
import hashlib
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG_DIR

pytestmark = pytest.mark.gpu
H = 256


def _dw2_once(mb, q, plans=None):
    if plans is not None:
        os.environ["SATRL_DW2_PLANS"] = plans
    sys.path.insert(0, PKG_DIR)
    from satrl.ppo import FusedMinibatch, PPOLearner
    from satrl.trainer import args_param
    torch.cuda.set_device(0)
    torch.manual_seed(3)
    args = args_param(hidden_width=H, mini_batch_size=mb, batch_size=8192, chkpt_dir="/tmp")
    args.state_dim, args.action_dim, args.max_action = 18, 3, 1.6
    L = PPOLearner(args, "pursuer", device="cuda:0", use_graph=False)
    st = FusedMinibatch(L, mb, 1, use_graph=False, kx=False)     # the library GEMM path itself
    g = torch.Generator(device="cuda:0").manual_seed(9)
    n = 2 * mb * H
    H1 = torch.rand(n, device="cuda:0", generator=g) * 2 - 1
    dZ2 = torch.randn(n, device="cuda:0", generator=g) * 1e-3
    st._dw2(H1, dZ2, mb, st.S, -1)
    torch.cuda.synchronize()
    p2 = st.p2[:2 * st.S * H * H].cpu().numpy()
    q.put((hashlib.sha256(p2.tobytes()).hexdigest(), st.dw2_algo, st.dw2_source, st.dw2_kernel))


@pytest.mark.parametrize("mb", [512, 4096])
def test_dw2_bitwise_across_processes(mb):
    """Two fresh processes make the plan of the same shape and compute the
    same dW2 slabs bit for bit, with the table's solution."""
    ctx = mp.get_context("spawn")
    res = []
    for _ in range(2):
        q = ctx.Queue()
        p = ctx.Process(target=_dw2_once, args=(mb, q))
        p.start()
        res.append(q.get(timeout=300))
        p.join(timeout=60)
        assert p.exitcode == 0
    (h0, a0, s0, k0), (h1, a1, s1, k1) = res
    print(f"mb {mb}: solution {a0} ({s0}) {k0}")
    assert s0 == s1 == "table", "the committed dw2_plans.json has no usable entry for this shape"
    assert a0 == a1 and k0 == k1 and h0 == h1


def _dp_rank(rank, port, q):
    import torch.distributed as dist
    os.environ["SATRL_DW2_PLANS"] = "none"          # rank 0 tunes, rank 1 must take its choice
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        sys.path.insert(0, PKG_DIR)
        from satrl.ppo import PPOLearner
        from satrl.trainer import args_param
        torch.manual_seed(3)
        args = args_param(hidden_width=H, mini_batch_size=512, batch_size=8192, chkpt_dir="/tmp")
        args.state_dim, args.action_dim, args.max_action = 18, 3, 1.6
        L = PPOLearner(args, "pursuer", device="cuda:0", pg=dist.group.WORLD, use_graph=False)
        st = L.stepper(512)
        q.put((rank, st.dw2_algo, st.dw2_kernel, st.dw2_source))
    finally:
        dist.destroy_process_group()


def test_dp_ranks_pin_rank0_solution():
    """Under data parallelism every rank runs rank 0's dW2 solution (the
    configs[3] per-rank shape, 512 rows), whatever its own tuner would pick."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_dp_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (a, k, src) for r, a, k, src in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res[0][2] == "tuned" and res[1][2] == "rank0"
    assert res[0][:2] == res[1][:2]


def _split_update(split):
    sys.path.insert(0, PKG_DIR)
    from satrl.ppo import FusedMinibatch, PPOLearner
    from satrl.trainer import args_param
    torch.manual_seed(21)
    mb, B = 4096, 4096 * 17
    args = args_param(hidden_width=H, mini_batch_size=mb, batch_size=B, K_epochs=1, use_lr_decay=False,
                      chkpt_dir="/tmp")
    args.state_dim, args.action_dim, args.max_action = 18, 3, 1.6
    L = PPOLearner(args, "pursuer", device="cuda:0", graph_group=4, use_graph=True)
    L._steppers[mb] = FusedMinibatch(L, mb, 4, use_graph=True, split_chains=split, kx=False)
    g = torch.Generator(device="cuda:0").manual_seed(2)
    src = torch.zeros((B, 32), device="cuda:0")
    src[:, 0:18] = torch.randn((B, 18), device="cuda:0", generator=g)
    src[:, 18:21] = torch.rand((B, 3), device="cuda:0", generator=g) * 3.2 - 1.6
    src[:, 21:24] = -1.0 - torch.rand((B, 3), device="cuda:0", generator=g)
    src[:, 24] = torch.randn(B, device="cuda:0", generator=g)
    src[:, 25] = torch.randn(B, device="cuda:0", generator=g) * 5
    perm = torch.randperm(B, device="cuda:0", generator=g)
    L.update_packed(src, 0, perms=[perm])      # 4 graph groups of 4 + one eager minibatch
    torch.cuda.synchronize()
    return L.P.clone(), L.G.clone()


def test_split_chains_have_own_workspaces():
    """The actor and critic chains on two streams (split_chains) each get a
    hipBLASLt workspace of their own: two runs of 17 minibatch steps (graphed
    groups + an eager one) agree bit for bit, and with the fused chain within
    the fused step's tolerance."""
    p0, g0 = _split_update(True)
    p1, g1 = _split_update(True)
    assert torch.equal(p0, p1) and torch.equal(g0, g1)
    pf, _ = _split_update(False)
    assert torch.allclose(p0, pf, rtol=1e-4, atol=1e-5), (p0 - pf).abs().max().item()
