"""RCCL communicator on the caller's stream, for the per-minibatch gradient
all-reduce of the data-parallel update (SURVEY.md §8e collective (3);
the reference trains on one process and has no counterpart).

torch.distributed's ``nccl`` backend is RCCL on ROCm, but every c10d
collective runs on the process group's internal stream with event hand-offs
both ways and host-side work objects, so a minibatch step that contains one
cannot live in the same hipGraph as its kernels.  This module binds the
RCCL library torch itself loaded (``torch/lib/librccl.so``) through ctypes,
builds one communicator over the ranks of a process group (the unique id
travels over that group), and issues ``ncclAllReduce`` on the current HIP
stream -- so reduce -> all-reduce -> reduce -> Adam is one stream chain that
``torch.cuda.graph`` captures whole, RCCL kernels included (RCCL supports
stream capture).  Ring / tree all-reduce reduces every element once in a
fixed order and broadcasts it, so every rank receives identical bits.
"""
from __future__ import annotations

import ctypes as C
import os
import time

import torch

NCCL_UNIQUE_ID_BYTES = 128            # rccl.h:40
_NCCL_FLOAT32, _NCCL_FLOAT64 = 7, 8   # rccl.h:466-467 ncclDataType_t
_NCCL_SUM = 0                         # rccl.h:448 ncclRedOp_t
_NCCL_IN_PROGRESS = 7                 # ncclResult_t ncclInProgress


class CommError(RuntimeError):
    """A collective failed or stalled: the communicator has been aborted
    (ncclCommAbort), so the caller must not issue further collectives on it."""


class _UniqueId(C.Structure):
    _fields_ = [("internal", C.c_byte * NCCL_UNIQUE_ID_BYTES)]


_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        if not os.path.exists(path):
            path = "librccl.so"
        lib = C.CDLL(path)
        lib.ncclGetErrorString.restype = C.c_char_p
        lib.ncclGetUniqueId.argtypes = [C.POINTER(_UniqueId)]
        lib.ncclCommInitRank.argtypes = [C.POINTER(C.c_void_p), C.c_int, _UniqueId, C.c_int]
        lib.ncclAllReduce.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        lib.ncclCommDestroy.argtypes = [C.c_void_p]
        lib.ncclCommAbort.argtypes = [C.c_void_p]
        lib.ncclCommGetAsyncError.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
        _LIB = lib
    return _LIB


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: RCCL error {rc}: {_lib().ncclGetErrorString(rc).decode()}")


class Comm:
    """One RCCL communicator over the ranks of ``pg`` (an initialised
    torch.distributed group whose backend can broadcast a CPU/CUDA uint8
    tensor), on the current CUDA device."""

    def __init__(self, pg, device):
        import torch.distributed as dist
        self.device = torch.device(device)
        self.world = dist.get_world_size(pg)
        self.rank = dist.get_rank(pg)
        lib = _lib()
        uid = _UniqueId()
        if self.rank == 0:
            _check(lib.ncclGetUniqueId(C.byref(uid)), "ncclGetUniqueId")
        raw = torch.tensor(list(bytes(uid.internal)), dtype=torch.uint8)
        if dist.get_backend(pg) == "nccl":
            raw = raw.to(self.device)
        dist.broadcast(raw, src=dist.get_global_rank(pg, 0), group=pg)
        C.memmove(uid.internal, bytes(raw.cpu().tolist()), NCCL_UNIQUE_ID_BYTES)
        self._comm = C.c_void_p()
        with torch.cuda.device(self.device):
            _check(lib.ncclCommInitRank(C.byref(self._comm), self.world, uid, self.rank), "ncclCommInitRank")
        self._warm = set()

    def all_reduce_sum_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place SUM over the ranks on torch's current stream (capturable)."""
        if t.dtype == torch.float32:
            dt = _NCCL_FLOAT32
        elif t.dtype == torch.float64:
            dt = _NCCL_FLOAT64
        else:
            raise TypeError(f"unsupported dtype {t.dtype}")
        if not t.is_contiguous() or t.device != self.device:
            raise ValueError("all_reduce_sum_ needs a contiguous tensor on the communicator's device")
        stream = torch.cuda.current_stream(self.device).cuda_stream
        _check(_lib().ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), dt, _NCCL_SUM, self._comm,
                                    C.c_void_p(stream)), "ncclAllReduce")
        return t

    def warm(self, t: torch.Tensor):
        """Run one eager all-reduce of t's size and dtype before a capture:
        RCCL connects each algorithm/protocol lazily on first use, which must
        not happen inside a stream capture.  (t's contents are destroyed.)"""
        key = (t.numel(), t.dtype)
        if key in self._warm:
            return
        self.all_reduce_sum_(t)
        torch.cuda.synchronize(self.device)
        self._warm.add(key)

    def async_error(self) -> int:
        """ncclCommGetAsyncError: 0 (ok), 7 (in progress) or an error code."""
        if not self._comm:
            return 0
        err = C.c_int(0)
        rc = _lib().ncclCommGetAsyncError(self._comm, C.byref(err))
        return rc if rc not in (0, _NCCL_IN_PROGRESS) else err.value

    def wait(self, deadline_s: float, stream=None, poll_s: float = 0.001):
        """Host watchdog: block until the work queued so far on `stream`
        (default: the current one) has finished, polling
        ncclCommGetAsyncError meanwhile (wait_event)."""
        ev = torch.cuda.Event()
        ev.record(stream)
        self.wait_event(ev, deadline_s, poll_s)

    def wait_event(self, ev, deadline_s: float, poll_s: float = 0.001):
        """Block until `ev` (a recorded torch.cuda.Event) has completed,
        polling ncclCommGetAsyncError meanwhile.  An RCCL error, or no
        completion within deadline_s (a dead or stalled peer leaves this
        rank's all-reduce kernels waiting forever), aborts the communicator
        (ncclCommAbort ends its kernels) and raises CommError.  The update
        calls it between graph replays (FusedMinibatch.run keeps at most two
        replays queued ahead of it), so a lost peer is caught within a
        deadline of its replay, not after the whole update was queued."""
        t0 = time.monotonic()
        while not ev.query():
            err = self.async_error()
            if err not in (0, _NCCL_IN_PROGRESS):
                self.abort()
                raise CommError(f"RCCL asynchronous error {err}: {_lib().ncclGetErrorString(err).decode()}")
            if time.monotonic() - t0 > deadline_s:
                self.abort()
                raise CommError(f"collective stalled: no completion within {deadline_s:.0f} s (peer lost?)")
            time.sleep(poll_s)

    def abort(self):
        if self._comm:
            _lib().ncclCommAbort(self._comm)
            self._comm = C.c_void_p()

    def destroy(self):
        if self._comm:
            _lib().ncclCommDestroy(self._comm)
            self._comm = C.c_void_p()


def abort_all():
    """ncclCommAbort every communicator of this process (the failure path)."""
    for c in list(_COMMS.values()):
        try:
            c.abort()
        except Exception:                          # noqa: BLE001 -- best effort on the way out
            pass


_COMMS = {}


def for_group(pg, device):
    """The process-wide RCCL communicator of (pg, device), or None when the
    group's backend is not nccl (gloo in the CPU tests) or SATRL_DP_GRAPH=0."""
    if pg is None or os.environ.get("SATRL_DP_GRAPH", "1") == "0":
        return None
    import torch.distributed as dist
    if dist.get_backend(pg) != "nccl":
        return None
    device = torch.device(device)
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    key = (id(pg), str(device))
    if key not in _COMMS:
        _COMMS[key] = Comm(pg, device)
    return _COMMS[key]
