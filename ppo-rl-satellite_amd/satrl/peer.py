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

Its grid is at most one workgroup per CU (satrl_peer_blocks, the minimum
over the ranks so every rank launches the same grid), and every wait for a
peer's value is bounded by the data-parallel timeout (SATRL_DP_TIMEOUT_S):
a rank that stops makes the others' calls give up and set an error word,
which ``check`` reads between graph replays (FusedMinibatch.run) and after
the update.  ``reset`` re-arms every rank's buffer after a barrier.
"""
from __future__ import annotations

import ctypes as C
import weakref

import torch

from . import _lib
from . import dist as _dist
from ._lib import check, ptr, stream_ptr

HANDLE_BYTES = 64            # SATRL_PEER_HANDLE_BYTES
MAX_WORLD = 8                # SATRL_PEER_MAX_WORLD


class PeerError(RuntimeError):
    """A peer's value never arrived within the kernel's bounded wait."""


def _release(lib, opened, own):
    """Unmap the peers' buffers and free this rank's (PeerComm.close and the
    finalizer of a PeerComm that was never closed)."""
    for p in opened:
        lib.satrl_peer_close(p)
    opened.clear()
    if own.value:
        lib.satrl_peer_free(own)
        own.value = None


class PeerComm:
    """Exchange buffers of `n`-float all-reduces over the ranks of `pg` (an
    initialised torch.distributed group; its backend only carries the IPC
    handles).  Every rank constructs it with the same n and H, in the same
    order."""

    def __init__(self, pg, n, device, H, timeout_s=None):
        import torch.distributed as dist
        self.pg = pg
        self.world = dist.get_world_size(pg)
        self.rank = dist.get_rank(pg)
        if not 1 <= self.world <= MAX_WORLD:
            raise ValueError(f"peer all-reduce supports 1..{MAX_WORLD} ranks, got {self.world}")
        self.device = torch.device(device)
        self.timeout_s = float(_dist.dp_timeout_s() if timeout_s is None else timeout_s)
        lib = _lib.lib()
        nbytes = C.c_int64()
        check(lib.satrl_peer_buffer_bytes(int(n), self.world, C.byref(nbytes)), "satrl_peer_buffer_bytes")
        self.n, self.nbytes = int(n), nbytes.value
        own = C.c_void_p()
        handle = (C.c_ubyte * HANDLE_BYTES)()
        blocks = C.c_int()
        with torch.cuda.device(self.device):
            check(lib.satrl_peer_blocks(int(H), C.byref(blocks)), "satrl_peer_blocks")
            check(lib.satrl_peer_alloc(self.nbytes, C.byref(own), handle), "satrl_peer_alloc")
        self._own = own
        self._opened = []
        self._fin = weakref.finalize(self, _release, lib, self._opened, own)
        gathered = [None] * self.world
        dist.all_gather_object(gathered, (bytes(handle), blocks.value), group=pg)
        self.blocks = min(b for _, b in gathered)            # the same grid on every rank
        ptrs = []
        with torch.cuda.device(self.device):
            for r, (h, _) in enumerate(gathered):
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
        check(_lib.lib().satrl_ppo_allreduce_peer(int(H), int(mb), self.world, self.rank, C.cast(self.bufs, C.c_void_p),
                                                  ptr(G), ptr(nsq), ptr(steps), self.blocks, self.timeout_s,
                                                  stream_ptr()), "satrl_ppo_allreduce_peer")
        return G

    def error(self, stream=None) -> int:
        """The sticky error word, after the work queued on `stream` (default:
        the current stream, which the read drains)."""
        err = C.c_uint64()
        check(_lib.lib().satrl_peer_error(self._own, C.byref(err), stream_ptr(stream)), "satrl_peer_error")
        return int(err.value)

    def _raise(self):
        raise PeerError("peer all-reduce: a peer's granule never arrived within "
                        f"{self.timeout_s:g} s (a rank stalled or died); PeerComm.reset re-arms the buffers")

    def check(self):
        if self.error():
            self._raise()

    def wait_event(self, ev, poll_s: float = 0.001):
        """The watchdog between graph replays (FusedMinibatch.run): wait for
        `ev` (recorded after a replay) by polling it against a host deadline,
        then read the error word on a side stream that waits for nothing, so
        the replays queued behind `ev` keep running (reading it on the compute
        stream would drain them).  Every wait in the kernel is bounded by
        timeout_s, and after one call fails the later ones return at once, so
        a replay with a lost peer ends within about timeout_s: the host
        deadline is twice that plus a margin."""
        import time
        t0, limit = time.monotonic(), 2.0 * self.timeout_s + 30.0
        while not ev.query():
            if time.monotonic() - t0 > limit:
                raise PeerError(f"peer all-reduce: replay not complete after {limit:.0f} s (GPU stalled?)")
            time.sleep(poll_s)
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
        if self.error(self._side):
            self._raise()

    _side = None

    def reset(self):
        """Re-arm after a failure (a collective call): a barrier, so every rank
        has stopped queueing calls; each rank drains its device, so none of
        its kernels still pushes into a peer's slots; a second barrier, so no
        buffer is zeroed while any rank's kernel may still write into it; then
        every rank zeroes its own buffer (counters, slots, error word) and a
        third barrier holds every rank until all buffers are re-armed."""
        import torch.distributed as dist
        dist.barrier(group=self.pg)
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.pg)
        check(_lib.lib().satrl_peer_reset(self._own, self.nbytes, stream_ptr()), "satrl_peer_reset")
        dist.barrier(group=self.pg)

    def close(self):
        self._fin()
