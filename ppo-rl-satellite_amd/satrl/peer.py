"""Peer (IPC / xGMI) gradient all-reduce for the data-parallel update: the
alternative to RCCL's ncclAllReduce + satrl_ppo_reduce_dp (include/
satrl_peer.h).  SURVEY.md §8e collective (3); the reference trains in one
process and has no counterpart.

Every rank allocates one exchange buffer (uncached device memory), sends its
IPC handle to the others over the process group, and maps theirs.  A call
(satrl_ppo_allreduce_peer) is one kernel on the caller's stream: it sums
each slice of G once, in rank order, divides by the world size and hands
the result to every rank, so every rank holds identical bits; it then writes
reduce_dp's squared-norm partials and advances the step counters.  It holds
no host state between calls, so it lives inside the update's hipGraphs like
the kernels around it.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from ._lib import check, ptr, stream_ptr

HANDLE_BYTES = 64            # SATRL_PEER_HANDLE_BYTES
MAX_WORLD = 8                # SATRL_PEER_MAX_WORLD


class PeerError(RuntimeError):
    """A peer's value never arrived within the kernel's bounded wait."""


class PeerComm:
    """Exchange buffers of `n`-float all-reduces over the ranks of `pg` (an
    initialised torch.distributed group; its backend only carries the IPC
    handles).  Every rank constructs it with the same n, in the same order."""

    def __init__(self, pg, n, device):
        import torch.distributed as dist
        self.pg = pg
        self.world = dist.get_world_size(pg)
        self.rank = dist.get_rank(pg)
        if not 1 <= self.world <= MAX_WORLD:
            raise ValueError(f"peer all-reduce supports 1..{MAX_WORLD} ranks, got {self.world}")
        self.device = torch.device(device)
        lib = _lib.lib()
        nbytes = C.c_int64()
        check(lib.satrl_peer_buffer_bytes(int(n), self.world, C.byref(nbytes)), "satrl_peer_buffer_bytes")
        self.n = int(n)
        own = C.c_void_p()
        handle = (C.c_ubyte * HANDLE_BYTES)()
        with torch.cuda.device(self.device):
            check(lib.satrl_peer_alloc(nbytes.value, C.byref(own), handle), "satrl_peer_alloc")
        self._own = own
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(handle), group=pg)
        self._opened = []
        ptrs = []
        with torch.cuda.device(self.device):
            for r, h in enumerate(handles):
                if r == self.rank:
                    ptrs.append(own.value)
                    continue
                p = C.c_void_p()
                hb = (C.c_ubyte * HANDLE_BYTES).from_buffer_copy(h)
                check(lib.satrl_peer_open(hb, C.byref(p)), "satrl_peer_open")
                self._opened.append(p)
                ptrs.append(p.value)
        self.bufs = (C.c_void_p * self.world)(*ptrs)
        dist.barrier(group=pg)                       # every rank mapped every buffer before any call

    def all_reduce_dp_(self, H, mb, G, nsq, steps):
        """G <- (sum over ranks) / world, identical on every rank, and
        reduce_dp's norm partials / step counters (satrl_ppo_allreduce_peer),
        on the current stream (capturable)."""
        check(_lib.lib().satrl_ppo_allreduce_peer(int(H), int(mb), self.world, self.rank, C.cast(self.bufs, C.c_void_p), ptr(G),
                                                  ptr(nsq), ptr(steps), stream_ptr()), "satrl_ppo_allreduce_peer")
        return G

    def error(self) -> int:
        err = C.c_uint64()
        check(_lib.lib().satrl_peer_error(self._own, C.byref(err)), "satrl_peer_error")
        return int(err.value)

    def check(self):
        if self.error():
            raise PeerError("peer all-reduce: a peer's granule never arrived (a rank stalled or died)")

    def close(self):
        lib = _lib.lib()
        for p in self._opened:
            lib.satrl_peer_close(p)
        self._opened = []
        if self._own:
            lib.satrl_peer_free(self._own)
            self._own = C.c_void_p()
