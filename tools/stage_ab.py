#!/usr/bin/env python3
"""Development tool (not shipped, not a test): graph replays with the next
group's rows staged on a forked branch against the stage at the head of
each group's own graph (serial, the product), at the bench's graph group
(64): per-minibatch time over epochs of `reps` replays.  Needs the forked
variant of FusedMinibatch (commit history, round 5: two graphs, two stage
buffers, `_stage_next`); kept for the record.
Usage: python tools/stage_ab.py [H] [mb] [replays per epoch]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
from satrl import _lib  # noqa: E402
from satrl._lib import check, ptr, stream_ptr  # noqa: E402
from satrl.ppo import FusedMinibatch, PPOLearner  # noqa: E402
from satrl.trainer import args_param  # noqa: E402


def serial_group_dev(self, src, i):
    mb, G = self.mb, self.group
    check(_lib.lib().satrl_ppo_stage(G * mb, ptr(src), ptr(self.perm_buf), ptr(self.grp),
                                     ptr(self.stage_bufs[i]), stream_ptr()), "satrl_ppo_stage")
    check(_lib.lib().satrl_ppo_group_advance(ptr(self.grp), stream_ptr()), "satrl_ppo_group_advance")
    stage = self.stage_bufs[i]

    def chain(net):
        for k in range(G):
            self._net_step(stage[k * mb:(k + 1) * mb], None, mb, net)
    self._chains(chain)


def time_it(H, mb, reps, serial, n=6, G=64):
    B = G * reps * mb
    a = args_param(hidden_width=H, mini_batch_size=mb, batch_size=B, chkpt_dir="/tmp")
    L = PPOLearner(a, "pursuer", graph_group=G)
    g = torch.Generator(device="cuda").manual_seed(0)
    src = torch.randn((B, 32), device="cuda", generator=g)
    src[:, 21:24] = -1.0 - torch.rand((B, 3), device="cuda", generator=g)
    st = FusedMinibatch(L, mb, G)
    if serial:
        st._group_dev = serial_group_dev.__get__(st)
        st._stage_next = (lambda src, i: None)
    perm = torch.randperm(B, device="cuda", generator=g)
    L.sync_w2t()
    for _ in range(2):
        st.run(src, perm)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        st.run(src, perm)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (n * B // mb)


if __name__ == "__main__":
    H = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    mb = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    for r in range(2):
        for serial in (False, True):
            print(f"H {H} mb {mb} x{reps} groups of 64: {'serial stage ' if serial else 'forked stage '}: "
                  f"{time_it(H, mb, reps, serial):7.2f} us per minibatch step", flush=True)
