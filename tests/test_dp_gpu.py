"""Data-parallel minibatch step on the GPU: two ranks (gloo over CUDA
tensors, both on cuda:0) each step their half of a minibatch through the
DP path of FusedMinibatch (reduce mode 1 -> all-reduce of G -> mode 2 ->
Adam).  Both ranks must end bitwise identical, and equal (within the fused
step's tolerance) to one process stepping the whole minibatch."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG_DIR

pytestmark = pytest.mark.gpu

H, MB, B = 64, 256, 4096
TESTS_DIR = os.path.dirname(os.path.abspath(__file__))


def _setup(pg, mb):
    sys.path.insert(0, PKG_DIR)
    from satrl.ppo import PPOLearner
    from satrl.trainer import args_param
    torch.manual_seed(11)
    args = args_param(hidden_width=H, mini_batch_size=mb, batch_size=B, chkpt_dir="/tmp")
    args.state_dim, args.action_dim, args.max_action = 18, 3, 1.6
    L = PPOLearner(args, "pursuer", device="cuda:0", pg=pg, use_graph=False)
    with torch.no_grad():
        for p in list(L.actor.parameters()) + list(L.critic.parameters()):
            p.add_(torch.randn_like(p) * 0.05)
    g = torch.Generator(device="cuda:0").manual_seed(0)
    src = torch.zeros((B, 32), device="cuda:0")
    src[:, 0:18] = torch.randn((B, 18), device="cuda:0", generator=g)
    src[:, 18:21] = torch.rand((B, 3), device="cuda:0", generator=g) * 3.2 - 1.6
    src[:, 21:24] = -1.0 - torch.rand((B, 3), device="cuda:0", generator=g)
    src[:, 24] = torch.randn(B, device="cuda:0", generator=g)
    src[:, 25] = torch.randn(B, device="cuda:0", generator=g) * 5
    idx = torch.randperm(B, device="cuda:0", generator=g)[:2 * MB]
    L.sync_w2t()
    return L, src, idx


def _rank(rank, port, q):
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        L, src, idx = _setup(dist.group.WORLD, MB)
        L.stepper(MB).step(src, idx[rank * MB:(rank + 1) * MB].contiguous())
        torch.cuda.synchronize()
        q.put((rank, L.G.cpu().numpy(), L.P.cpu().numpy(), L.W2T.cpu().numpy()))   # by value
    finally:
        dist.destroy_process_group()


def test_dp_step_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (torch.from_numpy(g), torch.from_numpy(p_), torch.from_numpy(w)))
               for r, g, p_, w in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    (g0, p0, w0), (g1, p1, w1) = res[0], res[1]
    assert torch.equal(g0, g1) and torch.equal(p0, p1) and torch.equal(w0, w1)
    # one process, the whole 2*MB minibatch
    L, src, idx = _setup(None, 2 * MB)
    L.stepper(2 * MB).step(src, idx)
    torch.cuda.synchronize()
    gref, pref = L.G.cpu(), L.P.cpu()
    assert (g0 - gref).abs().max().item() <= 2e-5 * gref.abs().max().item()
    assert torch.allclose(p0, pref, rtol=1e-5, atol=2e-7)


def _collect_rank(rank, port, q):
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        sys.path.insert(0, PKG_DIR)
        from satrl.trainer import VecTrainer, args_param
        args = args_param(batch_size=32 * 24, mini_batch_size=128, hidden_width=64, K_epochs=1, num_envs=32,
                          horizon=24, max_episode_steps=10, seed=1, rollout_graph_chunk=8, chkpt_dir="/tmp")
        tr = VecTrainer(args, flag=0, d_capture=15000.0, pg=dist.group.WORLD, env_offset=rank * 32)
        tr.collect()
        torch.cuda.synchronize()
        q.put((rank, tr.buf.obs.cpu().numpy(), tr.buf.rew.cpu().numpy(), tr.buf.act.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_rollout_is_sharding_invariant():
    """2 ranks x 32 envs (env ids 0-31 and 32-63) == 1 process x 64 envs, bitwise:
    noise is keyed by global env id and parameters are broadcast from rank 0."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_collect_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (o, rw, a) for r, o, rw, a in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sys.path.insert(0, PKG_DIR)
    from satrl.trainer import VecTrainer, args_param
    args = args_param(batch_size=64 * 24, mini_batch_size=128, hidden_width=64, K_epochs=1, num_envs=64, horizon=24,
                      max_episode_steps=10, seed=1, rollout_graph_chunk=8, chkpt_dir="/tmp")
    tr = VecTrainer(args, flag=0, d_capture=15000.0)
    tr.collect()
    torch.cuda.synchronize()
    obs, rew, act = tr.buf.obs.cpu().numpy(), tr.buf.rew.cpu().numpy(), tr.buf.act.cpu().numpy()
    import numpy as np
    for r in range(2):
        o, rw, a = res[r]
        assert np.array_equal(o, obs[:, 32 * r:32 * (r + 1)])
        assert np.array_equal(rw, rew[:, 32 * r:32 * (r + 1)])
        assert np.array_equal(a, act[:, 32 * r:32 * (r + 1)])


def _nccl_update_rank(port, q):
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        q.put(_graphed_update(dist.group.WORLD))
    finally:
        dist.destroy_process_group()


def _graphed_update(pg):
    """Two epochs of 16 minibatches (4 graph groups of 4) through
    PPOLearner.update_packed, with the update's hipGraphs on."""
    sys.path.insert(0, PKG_DIR)
    from satrl.ppo import PPOLearner
    from satrl.trainer import args_param
    torch.manual_seed(5)
    args = args_param(hidden_width=H, mini_batch_size=MB, batch_size=B, K_epochs=2, chkpt_dir="/tmp")
    args.state_dim, args.action_dim, args.max_action = 18, 3, 1.6
    L = PPOLearner(args, "pursuer", device="cuda:0", pg=pg, graph_group=4, use_graph=True)
    g = torch.Generator(device="cuda:0").manual_seed(2)
    src = torch.zeros((B, 32), device="cuda:0")
    src[:, 0:18] = torch.randn((B, 18), device="cuda:0", generator=g)
    src[:, 18:21] = torch.rand((B, 3), device="cuda:0", generator=g) * 3.2 - 1.6
    src[:, 21:24] = -1.0 - torch.rand((B, 3), device="cuda:0", generator=g)
    src[:, 24] = torch.randn(B, device="cuda:0", generator=g)
    src[:, 25] = torch.randn(B, device="cuda:0", generator=g) * 5
    perms = [torch.randperm(B, device="cuda:0", generator=g) for _ in range(2)]
    L.update_packed(src, 100, perms=perms)
    torch.cuda.synchronize()
    used = L.comm is not None and L.stepper(MB).graph is not None
    return used, L.P.cpu().numpy(), L.W2T.cpu().numpy()


def test_rccl_graphed_dp_update_world1():
    """The data-parallel update on an nccl (RCCL) group: the gradient
    all-reduce is issued by satrl.rccl on the compute stream and captured in
    the update's hipGraphs with the kernels.  At world size 1 it must equal
    the single-process update bitwise (mode 1 | all-reduce | reduce_dp ==
    mode 3 when nothing is added or divided)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = ctx.Process(target=_nccl_update_rank, args=(port, q))
    p.start()
    used, pd, wd = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert used, "the DP update did not run from a graph with the RCCL communicator"
    _, ps, ws = _graphed_update(None)
    assert (pd == ps).all() and (wd == ws).all()


def _global_mb_args(num_envs, **kw):
    sys.path.insert(0, PKG_DIR)
    from satrl.trainer import args_param
    return args_param(batch_size=num_envs * 24, mini_batch_size=256, hidden_width=64, K_epochs=2, num_envs=num_envs,
                      horizon=24, max_episode_steps=10, seed=4, rollout_graph_chunk=8, update_graph_group=2,
                      chkpt_dir="/tmp", **kw)


def _global_mb_rank(rank, port, q):
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        from satrl.trainer import VecTrainer
        tr = VecTrainer(_global_mb_args(32), flag=0, d_capture=15000.0, pg=dist.group.WORLD, env_offset=rank * 32)
        assert tr.mb_local == 128 and tr.global_minibatch == 256 and tr.sampler == "stratified"
        tr.iteration()
        torch.cuda.synchronize()
        q.put((rank, tr.learner.P.cpu().numpy(), float(tr.learner.steps[0].item())))
    finally:
        dist.destroy_process_group()


def test_global_minibatch_dp_equals_one_process():
    """dp_minibatch="global" (SURVEY.md §8e): 2 ranks x 32 envs, each stepping
    mb/2 = 128 rows of every global minibatch of 256, over a whole iteration
    (rollout, GAE, global advantage normalisation, 2 epochs x 6 minibatches)
    == one process x 64 envs with the same stratified sampler and mb 256:
    the same global minibatches, the same number of Adam steps, parameters
    within the fused step's bar (the gradient sums and the advantage moments
    add in another order)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_global_mb_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (P, st) for r, P, st in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert (res[0][0] == res[1][0]).all()
    sys.path.insert(0, PKG_DIR)
    from satrl.trainer import VecTrainer
    tr = VecTrainer(_global_mb_args(64, minibatch_sampler="stratified"), flag=0, d_capture=15000.0)
    assert tr.mb_local == 256
    tr.iteration()
    torch.cuda.synchronize()
    P1, steps1 = tr.learner.P.cpu().numpy(), float(tr.learner.steps[0].item())
    assert res[0][1] == steps1 == 2 * (64 * 24 // 256)
    import numpy as np
    diff = np.abs(res[0][0] - P1)
    print(f"global-minibatch DP vs one process: max |param diff| {diff.max():.3e} after {steps1:.0f} Adam steps")
    assert np.allclose(res[0][0], P1, rtol=1e-5, atol=2e-7 * steps1), diff.max()


def test_per_gpu_minibatch_variant_and_labels():
    """dp_minibatch="per_gpu" keeps the named variant: each rank steps the
    full mini_batch_size (global minibatch mb * W).  Single-process default:
    uniform sampler over the local table (the reference's distribution)."""
    sys.path.insert(0, PKG_DIR)
    from satrl.trainer import VecTrainer
    tr = VecTrainer(_global_mb_args(64), flag=0, d_capture=15000.0)
    assert tr.sampler == "uniform" and tr.mb_local == 256 and tr.global_minibatch == 256
    tr = VecTrainer(_global_mb_args(64, dp_minibatch="per_gpu"), flag=0, d_capture=15000.0)
    assert tr.mb_local == 256 and tr.global_minibatch == 256
    perm = tr.epoch_perm()
    assert torch.equal(torch.sort(perm).values, torch.arange(64 * 24, device=perm.device))
    tr = VecTrainer(_global_mb_args(64, minibatch_sampler="stratified"), flag=0, d_capture=15000.0)
    perm = tr.epoch_perm()
    assert torch.equal(torch.sort(perm).values, torch.arange(64 * 24, device=perm.device))
    # every minibatch holds mb/8 rows of each 8-env block
    blk = (perm % 64) // 8
    for k in range(64 * 24 // 256):
        assert torch.equal(torch.bincount(blk[k * 256:(k + 1) * 256], minlength=8),
                           torch.full((8,), 32, device=perm.device))


def test_rollout_sharding_invariant_at_full_size():
    """BASELINE configs[2]'s env count, H 256: one 16384-env rollout equals two
    8192-env shards (global env ids 0-8191 and 8192-16383, same seed) bit for
    bit -- obs, rewards, done flags, actions and log-probs over 24 steps with
    episodes ending and resetting in-kernel."""
    sys.path.insert(0, PKG_DIR)
    from satrl.trainer import VecTrainer, args_param

    def collect(n, offset):
        args = args_param(batch_size=n * 24, mini_batch_size=4096, hidden_width=256, K_epochs=1, num_envs=n,
                          horizon=24, max_episode_steps=9, seed=3, rollout_graph_chunk=8, chkpt_dir="/tmp")
        tr = VecTrainer(args, flag=0, d_capture=15000.0, env_offset=offset)
        tr.collect()
        torch.cuda.synchronize()
        b = tr.buf
        out = [x.cpu().numpy() for x in (b.obs, b.rew, b.done, b.act, b.logp)]
        del tr
        return out

    full = collect(16384, 0)
    halves = [collect(8192, 0), collect(8192, 8192)]
    import numpy as np
    for k, name in enumerate(("obs", "rew", "done", "act", "logp")):
        got = np.concatenate([halves[0][k], halves[1][k]], axis=1)
        assert np.array_equal(got, full[k]), name
    assert full[2].any()                                  # episodes did end inside the window


def test_comm_wait_deadline_and_async_error_raise():
    """The RCCL watchdog (satrl.rccl.Comm.wait / wait_event): a stream that
    does not finish within the deadline (a GPU spin standing in for a
    collective stuck on a lost peer) raises CommError, and so does an
    asynchronous communicator error; both abort the communicator (here: none
    made, so abort is a no-op)."""
    import ctypes as C

    from satrl import rccl
    c = rccl.Comm.__new__(rccl.Comm)
    c._comm = C.c_void_p()
    assert c.async_error() == 0
    torch.cuda._sleep(int(2e9))                       # ~1 s of GPU spin on the current stream
    with pytest.raises(rccl.CommError, match="stalled"):
        c.wait(0.05)
    torch.cuda.synchronize()
    c.wait(5.0)                                       # finished work: returns
    c.async_error = lambda: 3                         # ncclInternalError
    torch.cuda._sleep(int(2e8))
    with pytest.raises(rccl.CommError, match="asynchronous error"):
        c.wait(60.0)
    torch.cuda.synchronize()


def _peer_rank(rank, port, q):
    """World 2 on one device: the peer all-reduce (satrl_ppo_allreduce_peer,
    IPC-mapped buffers) against c10d's SUM / world + satrl_ppo_reduce_dp, on
    a raw gradient and through whole DP updates (eager and graph-replayed)."""
    import torch.distributed as dist
    os.environ["SATRL_DP_TIMEOUT_S"] = "30"           # the peer waits' bound: a stall fails, never hangs
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        sys.path.insert(0, PKG_DIR)
        import satrl._lib as _L
        from satrl.ppo import PPOLearner
        from satrl.trainer import args_param
        out = {}
        # (1) one raw gradient bucket: peer kernel vs gloo SUM + reduce_dp
        args = args_param(hidden_width=256, mini_batch_size=512, batch_size=B, chkpt_dir="/tmp", allreduce="peer")
        Lp = PPOLearner(args, "pursuer", device="cuda:0", pg=dist.group.WORLD, use_graph=False)
        assert Lp.peer is not None and Lp.comm is None
        g = torch.Generator(device="cuda:0").manual_seed(100 + rank)
        G0 = torch.randn(Lp.G.numel(), device="cuda:0", generator=g)
        st = Lp.stepper(512)
        nsq_p = torch.zeros_like(st.nsq[0])
        steps_p = torch.zeros(2, dtype=torch.float64, device="cuda:0")
        Gp = G0.clone()
        for _ in range(3):                                  # three calls: tags advance, buffers reused
            Gp.copy_(G0)
            Lp.peer.all_reduce_dp_(256, 512, Gp, nsq_p, steps_p)
        torch.cuda.synchronize()
        Gg = G0.clone().cpu()
        dist.all_reduce(Gg)
        Gg = Gg.cuda()
        nsq_g = torch.zeros_like(nsq_p)
        steps_g = torch.full((2,), 2.0, dtype=torch.float64, device="cuda:0")
        _L.check(_L.lib().satrl_ppo_reduce_dp(256, 512, -1, 2, _L.ptr(Gg), _L.ptr(nsq_g), _L.ptr(steps_g),
                                              _L.stream_ptr()), "satrl_ppo_reduce_dp")
        torch.cuda.synchronize()
        out["raw"] = (torch.equal(Gp, Gg), torch.equal(nsq_p, nsq_g), torch.equal(steps_p, steps_g), Gp.cpu().numpy())
        assert Lp.peer.error() == 0
        props = torch.cuda.get_device_properties(0)
        assert 1 <= Lp.peer.blocks <= props.multi_processor_count       # at most one spinning block per CU
        # (1b) a rank that skips a call: the other's waits run out (2 s here),
        # the error word is set and check raises; after reset on both ranks
        # the next call is bitwise the c10d path again
        from satrl.peer import PeerError
        if rank == 0:
            Lp.peer.timeout_s = 2.0
            Gp.copy_(G0)
            Lp.peer.all_reduce_dp_(256, 512, Gp, nsq_p, steps_p)
            try:
                Lp.peer.check()
                raise AssertionError("a missing peer was not reported")
            except PeerError:
                pass
            Lp.peer.timeout_s = 30.0
        dist.barrier()
        Lp.peer.reset()
        assert Lp.peer.error() == 0
        Gp.copy_(G0)
        steps_p.fill_(2.0)
        Lp.peer.all_reduce_dp_(256, 512, Gp, nsq_p, steps_p)
        torch.cuda.synchronize()
        out["reset"] = (torch.equal(Gp, Gg), torch.equal(nsq_p, nsq_g), torch.equal(steps_p, steps_g),
                        Lp.peer.error() == 0)
        # (1c) a rank that arrives LATE (after the other's deadline) rather than
        # never: the early rank's waits run out, it pushes no sum with a missing
        # term and flags every rank's buffer, so the late rank's call fails at
        # once (its own deadline is 30 s) instead of completing on partial sums
        import time
        Lp.peer.timeout_s = 2.0 if rank == 0 else 30.0
        dist.barrier()
        if rank == 1:
            time.sleep(5.0)
        t0 = time.monotonic()
        Gp.copy_(G0)
        Lp.peer.all_reduce_dp_(256, 512, Gp, nsq_p, steps_p)
        torch.cuda.synchronize()
        out["late"] = (time.monotonic() - t0, Lp.peer.error() != 0)
        Lp.peer.timeout_s = 30.0
        Lp.peer.reset()
        assert Lp.peer.error() == 0
        # (2) DP updates, H 64: peer path (graph-replayed and eager) vs the gloo path
        res = {}
        for mode, graph in (("peer", True), ("peer", False), ("rccl", False)):
            torch.manual_seed(11)
            a2 = args_param(hidden_width=H, mini_batch_size=MB, batch_size=B, chkpt_dir="/tmp", allreduce=mode,
                            K_epochs=2)
            L = PPOLearner(a2, "pursuer", device="cuda:0", pg=dist.group.WORLD, graph_group=2, use_graph=graph)
            gg = torch.Generator(device="cuda:0").manual_seed(7 + rank)
            src = torch.randn((B, 32), device="cuda:0", generator=gg)
            src[:, 21:24] = -1.0 - torch.rand((B, 3), device="cuda:0", generator=gg)
            L.sync_w2t()
            pg = torch.Generator(device="cuda:0").manual_seed(3)
            L.update_packed(src, 0.0, perms=[torch.randperm(B, device="cuda:0", generator=pg)[:5 * MB + 37]
                                             for _ in range(2)])
            torch.cuda.synchronize()
            res[(mode, graph)] = (L.P.clone(), L.M.clone(), L.V.clone(), L.steps.clone())
            if L.peer is not None:
                assert L.peer.error() == 0
                L.peer.close()
        same = [all(torch.equal(a, b) for a, b in zip(res[("peer", True)], res[k]))
                for k in (("peer", False), ("rccl", False))]
        out["update"] = (same, res[("peer", True)][0].cpu().numpy())
        Lp.peer.close()
        q.put((rank, out))
    except BaseException:
        import traceback
        q.put((rank, traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def test_peer_allreduce_world2_one_device():
    """satrl_ppo_allreduce_peer over two ranks on one GPU (IPC within the
    device): bitwise c10d's SUM / world and reduce_dp's norms and step
    counters on a raw gradient over three calls, bitwise identical on both
    ranks; a call one rank skips times out into the error word, and after
    PeerComm.reset the next call is bitwise right again; a rank that arrives
    after the other's deadline fails fast on the error word the other set in
    its buffer; whole DP updates (2 epochs of 5 minibatches + a ragged tail,
    graph-replayed and eager) bitwise equal to the gloo-all-reduce path."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ps = [ctx.Process(target=_peer_rank, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    import queue
    import time
    res, t_end = {}, time.monotonic() + 150
    while len(res) < 2 and time.monotonic() < t_end:
        try:
            r, v = q.get(timeout=2)
            assert not isinstance(v, str), f"rank {r}:\n{v}"
            res[r] = v
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in ps):
                break
    for p in ps:
        p.join(timeout=30)
        if p.exitcode is None:
            p.kill()
    assert len(res) == 2 and all(p.exitcode == 0 for p in ps), ([p.exitcode for p in ps], sorted(res))
    for r in (0, 1):
        eqG, eqN, eqS, _ = res[r]["raw"]
        assert eqG and eqN and eqS, (r, eqG, eqN, eqS)
        assert all(res[r]["reset"]), (r, res[r]["reset"])
        assert res[r]["late"][1], (r, "late peer: the failed call was not flagged on this rank")
        assert all(res[r]["update"][0]), (r, res[r]["update"][0])
    assert res[1]["late"][0] < 10.0, res[1]["late"]        # the late rank failed fast, not after its 30 s
    import numpy as np
    assert np.array_equal(res[0]["raw"][3], res[1]["raw"][3])
    assert np.array_equal(res[0]["update"][1], res[1]["update"][1])
