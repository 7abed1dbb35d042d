#!/usr/bin/env python3
"""Development tool (not shipped, not a test): upper bound of an L2 row
prefetch -- the in-graph step when every minibatch of a graph group reads
the group's FIRST staged rows (L2-warm after the first step, same XCD per
workgroup) against the product's fresh rows.  Timing only (wrong update).
Usage: python tools/rows_hot.py [H] [mb]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
from satrl import _lib  # noqa: E402
from satrl._lib import check, ptr, stream_ptr  # noqa: E402
from satrl.ppo import FusedMinibatch, PPOLearner  # noqa: E402
from satrl.trainer import args_param  # noqa: E402


def hot_group_dev(self, src):
    mb, G = self.mb, self.group
    check(_lib.lib().satrl_ppo_stage(G * mb, ptr(src), ptr(self.perm_buf), ptr(self.grp), ptr(self.stage),
                                     stream_ptr()), "satrl_ppo_stage")

    def chain(net):
        for k in range(G):
            self._net_step(self.stage[0:mb], None, mb, net)
    self._chains(chain)
    check(_lib.lib().satrl_ppo_group_advance(ptr(self.grp), stream_ptr()), "satrl_ppo_group_advance")


def time_it(H, mb, hot, n=20):
    B = 16 * mb
    a = args_param(hidden_width=H, mini_batch_size=mb, batch_size=B, chkpt_dir="/tmp")
    L = PPOLearner(a, "pursuer", graph_group=16)
    g = torch.Generator(device="cuda").manual_seed(0)
    src = torch.randn((B, 32), device="cuda", generator=g)
    src[:, 21:24] = -1.0 - torch.rand((B, 3), device="cuda", generator=g)
    st = FusedMinibatch(L, mb, 16)
    if hot:
        st._group_dev = hot_group_dev.__get__(st)
    perm = torch.randperm(B, device="cuda", generator=g)
    L.sync_w2t()
    for _ in range(3):
        st.run(src, perm)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        st.run(src, perm)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (n * 16)


if __name__ == "__main__":
    H = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    mb = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    for r in range(2):
        for hot in (False, True):
            print(f"H {H} mb {mb}: {'hot rows' if hot else 'product '}: {time_it(H, mb, hot):7.2f} us per step",
                  flush=True)
