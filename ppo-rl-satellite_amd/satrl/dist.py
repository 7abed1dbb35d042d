"""Data-parallel plumbing: one process per GPU, envs sharded
by global env id, and exactly four collectives -- the start-up parameter
broadcast, one all-reduce of (sum, sum of squares, count) of the advantages
per update, one all-reduce of the flat gradient per minibatch (both nets,
one bucket, before clipping so every rank clips identically), and the
episode-statistics sum.  Plain torch.distributed calls on whatever device
the tensors live on: RCCL over xGMI on the GPUs, gloo in the CPU tests.
(On the GPUs the per-minibatch gradient all-reduce goes through
satrl.rccl instead, on the compute stream, so that it is captured in the
update's hipGraphs.)
``pg=None`` means a single process (every function is then local).

Failure path: ``run_or_exit`` runs a multi-rank program and turns any
failure -- a collective error, a lost peer (gloo raises when its socket
closes; c10d times out after the group's timeout), or the RCCL watchdog of
satrl.rccl.Comm.wait (ncclCommGetAsyncError polling with a deadline) --
into ncclCommAbort of this process's communicators and a non-zero exit,
without restarting in place."""
from __future__ import annotations

import os
import sys
import traceback

import torch

EXIT_PEER_FAILURE = 3


def world_size(pg) -> int:
    if pg is None:
        return 1
    import torch.distributed as dist
    return dist.get_world_size(pg)


def rank(pg) -> int:
    if pg is None:
        return 0
    import torch.distributed as dist
    return dist.get_rank(pg)


def env_offset(pg, n_local: int) -> int:
    """First global env id of this rank (rank r owns [r*n, (r+1)*n))."""
    return rank(pg) * int(n_local)


def broadcast_(tensors, pg, src: int = 0):
    """Start-up: every rank takes rank src's parameters (in place)."""
    if pg is None:
        return
    import torch.distributed as dist
    for t in tensors:
        dist.broadcast(t, src=src, group=pg)


def broadcast_object(obj, pg, src: int = 0):
    """Rank src's picklable `obj` on every rank (start-up decisions such as
    the dW2 plan's solution)."""
    if pg is None:
        return obj
    import torch.distributed as dist
    box = [obj]
    dist.broadcast_object_list(box, src=dist.get_global_rank(pg, src), group=pg)
    return box[0]


def global_mean_std(local3: torch.Tensor, pg):
    """local3 = [sum, sum of squares, count] (f64) of this rank's advantages
    -> global mean and unbiased std (ppo_continuous.py:209-210 uses
    torch.std, i.e. n-1), both f64 tensors."""
    buf = local3.to(torch.float64).clone()
    if pg is not None:
        import torch.distributed as dist
        dist.all_reduce(buf, group=pg)
    s, s2, n = buf[0], buf[1], buf[2]
    mean = s / n
    var = (s2 - n * mean * mean) / (n - 1)
    return mean, var.clamp_min(0).sqrt()


def average_(flat: torch.Tensor, pg) -> torch.Tensor:
    """Per minibatch: every rank's gradient of its own minibatch mean ->
    the mean over ranks (= the gradient of the mean over all ranks' rows)."""
    if pg is not None:
        import torch.distributed as dist
        dist.all_reduce(flat, group=pg)
        flat.div_(world_size(pg))
    return flat


def sum_inplace_(flat: torch.Tensor, pg) -> torch.Tensor:
    """Per minibatch, c10d form: SUM of every rank's gradient in place (the
    division by the world size happens in satrl_ppo_reduce_dp)."""
    if pg is not None:
        import torch.distributed as dist
        dist.all_reduce(flat, group=pg)
    return flat


def sum_(t: torch.Tensor, pg) -> torch.Tensor:
    """Episode statistics: totals over ranks (returns a new tensor)."""
    out = t.clone()
    if pg is not None:
        import torch.distributed as dist
        dist.all_reduce(out, group=pg)
    return out


def dp_timeout_s() -> float:
    """Host deadline of one watched stretch of collectives (SATRL_DP_TIMEOUT_S,
    default 600 s)."""
    return float(os.environ.get("SATRL_DP_TIMEOUT_S", "600"))


def run_or_exit(fn, *args, world: int = 1, **kw):
    """fn(*args, **kw); in a multi-rank run any exception aborts the RCCL
    communicators and ends the process with EXIT_PEER_FAILURE (os._exit: the
    normal interpreter exit would run process-group teardown, which can
    block on a dead peer).  At world size 1 exceptions propagate."""
    if world <= 1:
        return fn(*args, **kw)
    try:
        return fn(*args, **kw)
    except BaseException as e:                   # noqa: BLE001 -- every failure ends the rank
        if isinstance(e, SystemExit) and not e.code:
            raise
        sys.stderr.write(f"[rank {os.environ.get('RANK', '?')}] data-parallel failure, aborting: {e!r}\n")
        traceback.print_exc()
        try:
            from . import rccl
            rccl.abort_all()
        except Exception:                        # noqa: BLE001
            pass
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(EXIT_PEER_FAILURE)
