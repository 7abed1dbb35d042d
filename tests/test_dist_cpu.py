"""Data-parallel plumbing (satrl.dist) with world_size 2 on the CPU (gloo):
the collectives the GPU path runs over RCCL, checked against the
single-process answer on the concatenated data."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_DIR


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    sys.path.insert(0, PKG_DIR)
    from satrl import dist as D
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    pg = dist.group.WORLD
    try:
        out = {}
        # advantages: rank-specific sizes and values
        rng = np.random.default_rng(100 + rank)
        adv = torch.tensor(rng.normal(rank, 2.0, 1000 + 37 * rank))
        local3 = torch.stack([adv.sum(), (adv * adv).sum(), torch.tensor(float(adv.numel()), dtype=torch.float64)])
        mean, std = D.global_mean_std(local3, pg)
        out["mean"], out["std"] = float(mean), float(std)
        # flat gradient averaging (in place)
        g = torch.arange(10, dtype=torch.float32) * (rank + 1)
        D.average_(g, pg)
        out["g"] = g.numpy()
        # start-up broadcast from rank 0
        p = torch.full((5,), float(rank + 7))
        D.broadcast_([p], pg)
        out["p"] = p.numpy()
        # episode statistics
        out["st"] = D.sum_(torch.tensor([1.0, 2.0 * rank, 3.0, rank], dtype=torch.float64), pg).numpy()
        out["off"] = D.env_offset(pg, 4096)
        out["ws"] = D.world_size(pg)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_dist_plumbing_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    allv = np.concatenate([np.random.default_rng(100 + r).normal(r, 2.0, 1000 + 37 * r) for r in range(2)])
    for r in range(2):
        o = res[r]
        assert o["mean"] == pytest.approx(allv.mean(), rel=1e-12)
        assert o["std"] == pytest.approx(allv.std(ddof=1), rel=1e-12)      # torch.std: unbiased
        assert np.array_equal(o["g"], (np.arange(10, dtype=np.float32) * 3) / 2)
        assert np.array_equal(o["p"], np.full(5, 7.0, dtype=np.float32))
        assert np.array_equal(o["st"], np.array([2.0, 2.0, 6.0, 1.0]))
        assert o["off"] == 4096 * r and o["ws"] == 2


def test_dist_single_process_is_local():
    sys.path.insert(0, PKG_DIR)
    from satrl import dist as D
    x = torch.tensor([1.0, 2.0, 3.0, 4.0], dtype=torch.float64)
    mean, std = D.global_mean_std(torch.stack([x.sum(), (x * x).sum(), torch.tensor(4.0, dtype=torch.float64)]), None)
    assert float(mean) == 2.5 and float(std) == pytest.approx(float(x.std()), rel=1e-15)
    g = torch.ones(3)
    assert D.average_(g, None) is g and torch.equal(g, torch.ones(3))
    assert D.rank(None) == 0 and D.world_size(None) == 1 and D.env_offset(None, 9) == 0


def test_stratified_minibatches_are_sharding_invariant():
    """satrl.trainer.stratified_epoch_perm: the global minibatches that W = 2,
    4 and 8 ranks step (each rank mb/W of its own rows, mapped back to global
    row ids) are exactly the W = 1 minibatches, in order, tail included."""
    import torch
    from satrl.trainer import stratified_epoch_perm
    T, N, mb = 7, 64, 48          # 448 rows, 9 full minibatches of 48 + a 16-row tail
    def gens():
        return {s: torch.Generator().manual_seed(1000 + s) for s in range(8)}
    ref = stratified_epoch_perm(T, N, 1, 0, mb, gens())
    assert sorted(ref.tolist()) == list(range(T * N))
    nfull = (T * N // 8) // (mb // 8)
    for W in (2, 4, 8):
        n = N // W
        parts = []
        for r in range(W):
            loc = stratified_epoch_perm(T, n, W, r, mb, gens())
            glob = (loc // n) * N + r * n + loc % n          # local row t*n + j -> global t*N + r*n + j
            parts.append(glob)
        m = mb // W
        for k in range(nfull):
            got = torch.cat([p[k * m:(k + 1) * m] for p in parts])
            assert torch.equal(torch.sort(got).values, torch.sort(ref[k * mb:(k + 1) * mb]).values), (W, k)
        got_tail = torch.cat([p[nfull * m:] for p in parts])
        assert torch.equal(torch.sort(got_tail).values, torch.sort(ref[nfull * mb:]).values)
