"""Live launch spans of the product kernels (satrl_span_probe, include/
satrl_ppo.h): the bench's kernel durations, measured in its own run.

While a ``SpanProbe`` is active, every launch of the rowpass, dW2, reduce,
Adam, policy / value and env-step kernels (eager, or captured into a graph
meanwhile) runs the kernel's SPAN instantiation, which adds one 16-B store
per wave at its exit: the wave's (start, exit) ``s_memrealtime`` pair
(100 MHz, one clock for the whole chip).  A launch's span is max(exit) -
min(start) over its waves: the time from its first wave's first instruction
to its last wave's exit, i.e. the kernel's duration without the dispatch
gaps around it.  A graph node keeps its record region, so after replays the
records are those of the last replay.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr

KINDS = {0: "rowpass", 1: "dw2", 2: "reduce", 3: "adam", 4: "policy_act", 5: "policy_value", 6: "env_step"}
TICK_US = 0.01                                   # s_memrealtime: 100 MHz


class SpanProbe:
    def __init__(self, nbytes=256 << 20, device="cuda"):
        self.buf = torch.empty(nbytes // 8, dtype=torch.int64, device=device)

    def __enter__(self):
        check(_lib.lib().satrl_span_probe(ptr(self.buf), self.buf.numel() * 8, stream_ptr()), "satrl_span_probe")
        return self

    def __exit__(self, *exc):
        _lib.lib().satrl_span_probe(None, 0, None)        # stop; the launch log stays readable
        return False

    def launches(self):
        """[(kind name, span_us, waves recorded / waves)] in launch (or capture) order."""
        torch.cuda.synchronize()
        lib = _lib.lib()
        rec = self.buf.cpu().numpy().view(np.uint64)
        out = []
        kind, off, waves = C.c_int(), C.c_int64(), C.c_int64()
        for i in range(int(lib.satrl_span_probe_launches())):
            check(lib.satrl_span_probe_launch(i, C.byref(kind), C.byref(off), C.byref(waves)),
                  "satrl_span_probe_launch")
            r = rec[off.value:off.value + 2 * waves.value].reshape(-1, 2)
            ok = r[:, 1] != 0
            span = float(r[ok, 1].max() - r[ok, 0].min()) * TICK_US if ok.any() else float("nan")
            out.append((KINDS.get(kind.value, str(kind.value)), span, int(ok.sum()), int(waves.value)))
        return out

    def raw(self):
        """[(kind name, first wave start, last wave exit)] in s_memrealtime ticks, launch order."""
        torch.cuda.synchronize()
        lib = _lib.lib()
        rec = self.buf.cpu().numpy().view(np.uint64)
        out = []
        kind, off, waves = C.c_int(), C.c_int64(), C.c_int64()
        for i in range(int(lib.satrl_span_probe_launches())):
            check(lib.satrl_span_probe_launch(i, C.byref(kind), C.byref(off), C.byref(waves)),
                  "satrl_span_probe_launch")
            r = rec[off.value:off.value + 2 * waves.value].reshape(-1, 2)
            ok = r[:, 1] != 0
            out.append((KINDS.get(kind.value, str(kind.value)), int(r[ok, 0].min()) if ok.any() else 0,
                        int(r[ok, 1].max()) if ok.any() else 0))
        return out

    def gaps(self, chain):
        """Mean idle time (us) between consecutive launches of a repeating kernel
        chain (e.g. ["rowpass", "dw2", "reduce", "adam"]): for each boundary
        "a->b", the next launch's first wave start minus the previous launch's
        last wave exit, over the log's launches in order (one graph replay's
        records); the span clock is one counter for the whole chip."""
        seq = [x for x in self.raw() if x[0] in chain and x[2] > 0]
        out = {}
        for (ka, _, ea), (kb, sb, _) in zip(seq, seq[1:]):
            out.setdefault(f"{ka}->{kb}", []).append((int(sb) - int(ea)) * TICK_US)
        return {k: {"mean_us": float(np.mean(v)), "median_us": float(np.median(v)), "n": len(v)}
                for k, v in out.items()}

    def summary(self):
        """{kind: {"launches", "avg_us", "median_us", "min_us", "max_us", "complete"}} over the log."""
        per = {}
        for k, us, got, n in self.launches():
            d = per.setdefault(k, {"spans": [], "complete": True})
            d["spans"].append(us)
            d["complete"] &= got == n
        out = {}
        for k, d in per.items():
            a = np.array(d["spans"], dtype=np.float64)
            out[k] = {"launches": int(a.size), "avg_us": float(a.mean()), "median_us": float(np.median(a)),
                      "min_us": float(a.min()), "max_us": float(a.max()), "complete": bool(d["complete"])}
        return out
