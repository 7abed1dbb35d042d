"""Gaussian PPO on PyTorch-ROCm + HIP rollout kernels.

Reference: qiaobeibei/PPO-RL-Satellite ppo_continuous.py.
  * ``Actor_Gaussian`` / ``Critic``       ppo_continuous.py:61-134 (same layer
    names, init, activations and checkpoint file names)
  * ``PPO_continuous``                     ppo_continuous.py:136-258, drop-in:
    choose_action / evaluate / update / lr_decay / save / load_checkpoint
  * ``PPOLearner``                          the batched engine used by the
    vectorised trainer: HIP Gaussian sampling, HIP GAE scan, and a
    hipGraph-captured minibatch step (actor and critic losses, backward,
    grad-norm clip, Adam) replayed over device-resident permutations.

The ``Actor_Beta`` policy (ppo_continuous.py:14-59) is outside the hot path
(policy_dist defaults to "Gaussian", CPPO_main.py:17).
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import dist as _dist
from . import rccl as _rccl
from ._lib import check, ptr, stream_ptr

LOG_SQRT_2PI = math.log(math.sqrt(2 * math.pi))
ENT_CONST = 0.5 + 0.5 * math.log(2 * math.pi)


def orthogonal_init(layer, gain=1.0):
    """ppo_continuous.py:10-12."""
    nn.init.orthogonal_(layer.weight, gain=gain)
    nn.init.constant_(layer.bias, 0)


class Actor_Gaussian(nn.Module):  # noqa: N801
    """ppo_continuous.py:61-101."""

    def __init__(self, args, agent_idx):
        super().__init__()
        self.agent_name = "agent_%s" % agent_idx
        self.chkpt_file = os.path.join(args.chkpt_dir, self.agent_name + "_actor_Gaussian")
        self.max_action = args.max_action
        self.fc1 = nn.Linear(args.state_dim, args.hidden_width)
        self.fc2 = nn.Linear(args.hidden_width, args.hidden_width)
        self.mean_layer = nn.Linear(args.hidden_width, args.action_dim)
        self.log_std = nn.Parameter(torch.zeros(1, args.action_dim))
        self.activate_func = [nn.ReLU(), nn.Tanh()][args.use_tanh]
        if args.use_orthogonal_init:
            orthogonal_init(self.fc1)
            orthogonal_init(self.fc2)
            orthogonal_init(self.mean_layer, gain=0.01)

    def forward(self, s):
        s = self.activate_func(self.fc1(s))
        s = self.activate_func(self.fc2(s))
        return self.max_action * torch.tanh(self.mean_layer(s))

    def get_dist(self, s):
        mean = self.forward(s)
        std = torch.exp(self.log_std.expand_as(mean))
        return torch.distributions.Normal(mean, std, validate_args=False)

    def save_checkpoint(self):
        torch.save({k: v.detach().cpu().clone() for k, v in self.state_dict().items()}, self.chkpt_file)

    def load_checkpoint(self):
        self.load_state_dict(torch.load(self.chkpt_file, weights_only=True, map_location="cpu"))


class Critic(nn.Module):
    """ppo_continuous.py:103-134."""

    def __init__(self, args, agent_idx):
        super().__init__()
        self.agent_name = "agent_%s" % agent_idx
        self.chkpt_file = os.path.join(args.chkpt_dir, self.agent_name + "_critic")
        self.fc1 = nn.Linear(args.state_dim, args.hidden_width)
        self.fc2 = nn.Linear(args.hidden_width, args.hidden_width)
        self.fc3 = nn.Linear(args.hidden_width, 1)
        self.activate_func = [nn.ReLU(), nn.Tanh()][args.use_tanh]
        if args.use_orthogonal_init:
            orthogonal_init(self.fc1)
            orthogonal_init(self.fc2)
            orthogonal_init(self.fc3)

    def forward(self, s):
        s = self.activate_func(self.fc1(s))
        s = self.activate_func(self.fc2(s))
        return self.fc3(s)

    def save_checkpoint(self):
        torch.save({k: v.detach().cpu().clone() for k, v in self.state_dict().items()}, self.chkpt_file)

    def load_checkpoint(self):
        self.load_state_dict(torch.load(self.chkpt_file, weights_only=True, map_location="cpu"))


# ---------------------------------------------------------------------------
# HIP kernels (include/satrl_rollout.h)
# ---------------------------------------------------------------------------
def gae(rew, done, values, gamma, lamda, adv_out=None, vt_out=None):
    """ppo_continuous.py:198-208 as a per-env reverse scan.

    rew f32 [T,N], done u8 [T,N], values f32 [T+1,N] -> adv, v_target f32 [T,N].
    A flat reference buffer of B transitions is the case N = 1."""
    T, N = rew.shape
    _lib.require_cuda(rew, torch.float32, (T, N), "rew")
    _lib.require_cuda(done, torch.uint8, (T, N), "done")
    _lib.require_cuda(values, torch.float32, (T + 1, N), "values")
    adv_out = torch.empty_like(rew) if adv_out is None else adv_out
    vt_out = torch.empty_like(rew) if vt_out is None else vt_out
    check(_lib.lib().satrl_gae(T, N, ptr(rew), ptr(done), ptr(values), float(gamma), float(lamda), ptr(adv_out),
                               ptr(vt_out), stream_ptr()), "satrl_gae")
    return adv_out, vt_out


def gaussian_sample(mean, log_std, max_action, seed, agent, env_offset, step, act_out=None, logp_out=None,
                    step_base=None):
    """choose_action (ppo_continuous.py:184-188) for a batch, counter-based RNG."""
    N = mean.shape[0]
    _lib.require_cuda(mean, torch.float32, (N, 3), "mean")
    log_std = log_std.reshape(-1)
    _lib.require_cuda(log_std, torch.float32, (3,), "log_std")
    act_out = torch.empty_like(mean) if act_out is None else act_out
    logp_out = torch.empty_like(mean) if logp_out is None else logp_out
    check(_lib.lib().satrl_gaussian_sample(N, ptr(mean), ptr(log_std), float(max_action), int(seed) & (2**64 - 1),
                                           int(agent), int(env_offset), int(step), ptr(step_base), ptr(act_out),
                                           ptr(logp_out), stream_ptr()), "satrl_gaussian_sample")
    return act_out, logp_out


def policy_act(H, obs, P0, P1, max_action, seed, env_offset, step, act0, logp0, act1=None, logp1=None,
               step_base=None):
    """Both agents' choose_action for a batch of observations on the fused
    MLP kernel (satrl_policy_act): P0/P1 are the pursuer's / evader's flat
    parameter buffers (PPOLearner.P), agent ids 0 / 1 in the noise key."""
    N = obs.shape[0]
    _lib.require_cuda(obs, torch.float32, (N, 18), "obs")
    for t, nm in ((act0, "act0"), (logp0, "logp0")) + (((act1, "act1"), (logp1, "logp1")) if P1 is not None else ()):
        _lib.require_cuda(t, torch.float32, (N, 3), nm)
    check(_lib.lib().satrl_policy_act(int(H), N, ptr(obs), ptr(P0), ptr(P1), float(max_action),
                                      int(seed) & (2**64 - 1), int(env_offset), int(step), ptr(step_base), ptr(act0),
                                      ptr(logp0), ptr(act1), ptr(logp1), stream_ptr()), "satrl_policy_act")


def policy_value(H, obs, P, v_out):
    """critic(obs) on the fused MLP kernel (satrl_policy_value)."""
    N = obs.shape[0]
    _lib.require_cuda(obs, torch.float32, (N, 18), "obs")
    check(_lib.lib().satrl_policy_value(int(H), N, ptr(obs), ptr(P), ptr(v_out), stream_ptr()), "satrl_policy_value")
    return v_out


def moments(x, out=None):
    out = torch.zeros(2, dtype=torch.float64, device=x.device) if out is None else out
    x = x.reshape(-1)
    check(_lib.lib().satrl_moments(x.numel(), ptr(x), ptr(out), stream_ptr()), "satrl_moments")
    return out


# ---------------------------------------------------------------------------
# fused minibatch step (ppo_continuous.py:213-239), include/satrl_ppo.h
# ---------------------------------------------------------------------------
OFF_NAMES = ["W2", "W1", "b2", "W3a", "b3a", "ls", "W3c", "b3c", "total"]


def ppo_layout(H):
    off = (C.c_int64 * 9)()
    check(_lib.lib().satrl_ppo_layout(int(H), off), "satrl_ppo_layout")
    return dict(zip(OFF_NAMES, [int(v) for v in off]))


def w2x_floats(H):
    """f32 elements of the fc2 operand image (satrl_ppo_w2x_floats)."""
    n = int(_lib.lib().satrl_ppo_w2x_floats(int(H)))
    if n <= 0:
        raise ValueError(f"hidden width {H} not supported")
    return n


def w2x_image(W2, H):
    """Host statement of satrl_ppo_w2x_sync: the fc2 operand image of the two
    nets' fc2.weight W2 (flat [2*H*H] f32), the f32 fc2.weight^T per net."""
    return W2.reshape(2, H, H).transpose(1, 2).contiguous().reshape(-1)


def w2x_decode(img, H):
    """fc2.weight^T per net [2, H, H] f32 from an operand image."""
    return img.view(2, H, H)


def rowpass_exchange_check(stream=None, timeout_s=None):
    """satrl_ppo_rowpass_error (include/satrl_ppo.h): waits for the stream (at
    most timeout_s of host time, default the DP watchdog's deadline
    SATRL_DP_TIMEOUT_S: a stream stuck behind a dead peer's collective raises
    NativeError instead of hanging); raises RuntimeError if a column-split
    short rowpass launch timed out waiting for the other workgroups of its
    group (its outputs, hence this update, are invalid), after the library has
    re-armed the exchange state."""
    L = _lib.lib()
    if _lib.LIB_PATH != _lib._PRODUCT_LIB and not hasattr(L, "satrl_ppo_rowpass_error"):
        return                               # (an older development build: A/B only)
    e = C.c_int(0)
    t = _dist.dp_timeout_s() if timeout_s is None else float(timeout_s)
    check(L.satrl_ppo_rowpass_error(C.byref(e), t, stream_ptr(stream)), "satrl_ppo_rowpass_error")
    if e.value:
        raise RuntimeError("satrl_ppo_rowpass_kx: a column-split exchange timed out (its workgroups were not "
                           "resident together); the update is invalid")


def uses_column_split(H, mb, B):
    """True when an update of B rows in minibatches of mb may run the
    column-split short rowpass (H = 256, a full or ragged-tail minibatch of at
    most 1024 rows; ppo_kernels.hip cs_fits): only such updates need
    rowpass_exchange_check."""
    mb = min(int(mb), int(B))
    tail = int(B) % mb if mb > 0 else 0
    return H == 256 and mb > 0 and (mb <= 1024 or 0 < tail <= 1024)


class FusedMinibatch:
    """One PPO minibatch step for actor + critic on shared rows:
    satrl_ppo_rowpass (gather, MLP forward/backward on f32 MFMA, losses),
    satrl_ppo_dw2 (the dW2 weight gradient, split-K), satrl_ppo_reduce and
    satrl_ppo_adam, both nets per launch.  The actor and
    critic steps share nothing but the rows (ppo_continuous.py:216-239 runs
    two independent optimisers); with ``split_chains`` they run as two
    per-net chains on two streams (the critic on a side stream, fork/join per
    group).  Under data parallelism both nets' gradients travel in one
    all-reduce.  Groups of ``group`` minibatches are captured into a hipGraph
    and replayed over [group, mb] blocks of a device permutation."""

    def __init__(self, learner, mb, group, use_graph=True, split_chains=False):
        self.L = learner
        self.mb = int(mb)
        self.group = int(group)
        self.use_graph = use_graph
        # dW2 (the fc2 weight gradient dZ2^T H1), hand-written at every width:
        # H = 64 (configs[1]): the rowpass multiplies each block's dW2 partial
        # out of LDS itself (satrl_ppo_rowpass_dw2), bitwise the dw2_kernel's
        # one-chunk splits, so a minibatch step is three launches;
        # H = 256: the rowpass writes H1 / dZ2 as k-packed bf16 planes and dW2
        # runs on the split-bf16 MFMA from them (satrl_ppo_rowpass_kx /
        # satrl_ppo_dw2_kx), for every minibatch size (16-row rowpass blocks up
        # to 1024 rows: configs[3]'s per-rank minibatch, ragged tails);
        # H = 128: f32 rows and dw2_kernel (satrl_ppo_dw2)
        self.fused_dw2 = learner.H == 64
        self.kx_on = learner.H == 256
        self.kx_elems = 0
        # two concurrent per-net chains: measured no faster than one fused chain at
        # H = 256 / 64, mb = 4096 on MI355X (the chains run in lockstep), so off by default
        self.split = bool(split_chains) and learner.pg is None
        H, dev = learner.H, learner.device
        nwg, nblk = C.c_int64(), C.c_int64()
        check(_lib.lib().satrl_ppo_sizes(H, self.mb, C.byref(nwg), C.byref(nblk)), "satrl_ppo_sizes")
        self.nwg, self.nblk = nwg.value, nblk.value
        self.S = self.splits(learner.H, self.mb)
        f32 = dict(dtype=torch.float32, device=dev)
        # f32 H1 / dZ2 rows: satrl_ppo_rowpass (the roofline's rowpass timing,
        # tests) and the H = 128 dW2; the H = 256 step hands them over as planes
        self.H1 = torch.empty(2 * self.mb * H, **f32)
        self.dZ2 = torch.empty(2 * self.mb * H, **f32)
        if self.kx_on:
            self.kx_elems = int(_lib.lib().satrl_ppo_kx_elems(H, self.mb))
            self.H1x = torch.empty(self.kx_elems, dtype=torch.int16, device=dev)
            self.dZ2x = torch.empty(self.kx_elems, dtype=torch.int16, device=dev)
        self.ptail = torch.empty(self.nwg * (6 * H + 12), **f32)
        self.pw1 = torch.empty(self.nwg * 2 * H * 20, **f32)
        # sized for the largest split count any minibatch size can produce, so
        # a ragged tail minibatch whose S exceeds the full minibatch's never
        # writes past the slabs
        # (the capacity is fixed here: the launch guard below compares against
        # it, not against max_splits(), which follows a later change of self.S)
        self.p2_splits = self.max_splits(H)
        self.p2 = torch.empty(2 * self.p2_splits * H * H, **f32)
        self.nsq = torch.zeros((2, 2 * self.nblk), dtype=torch.float64, device=dev)   # one per chain
        self.idx = torch.zeros((self.group, self.mb), dtype=torch.int64, device=dev)
        # the rows of one group of minibatches, gathered contiguously once per
        # group (one index_select) so rowpass reads them without an index hop
        self.stage = torch.empty((self.group * self.mb, 32), **f32)
        self.side = torch.cuda.Stream(device=dev) if self.split and torch.cuda.is_available() else None
        self.graph = None
        self._src_ptr = None
        # graph replays walk the epoch's permutation through a device group
        # counter (satrl_ppo_stage / satrl_ppo_group_advance): no host copy
        # or host round trip between groups
        self.perm_buf = None
        self.grp = torch.zeros(1, dtype=torch.int64, device=dev)
        if learner.pg is not None and _dist.world_size(learner.pg) > 1 and torch.cuda.is_available():
            # every rank's first step of this shape starts together (a rank
            # still setting up must not run into the peer all-reduce's bounded
            # wait)
            import torch.distributed as dist
            torch.cuda.synchronize()
            dist.barrier(group=learner.pg)

    def rowpass(self, src, idx, mb=None, net=-1):
        """satrl_ppo_rowpass alone (a pure function of src, idx and the
        parameters: bench.py times it on its own for the roofline).  idx None:
        rows 0..mb-1 of src.  net -1: both nets in one launch."""
        L = self.L
        H = L.H
        mb = self.mb if mb is None else int(mb)
        n = 2 * mb * H
        H1, dZ2 = self.H1[:n], self.dZ2[:n]
        check(_lib.lib().satrl_ppo_rowpass(H, mb, int(net), ptr(src), None if idx is None else ptr(idx), ptr(L.P),
                                           ptr(L.W2T), float(L.epsilon), float(L.entropy_coef), float(L.max_action),
                                           ptr(H1), ptr(dZ2), ptr(self.ptail), ptr(self.pw1), stream_ptr()),
                  "satrl_ppo_rowpass")
        return H1, dZ2

    def kx(self, mb):
        """True when a minibatch of mb rows takes the k-packed split-bf16 dW2
        path (H = 256, every minibatch size)."""
        return self.kx_on

    def rowpass_kx(self, src, idx, mb=None, net=-1):
        """satrl_ppo_rowpass_kx: the rowpass with H1 / dZ2 written as k-packed
        bf16 planes into self.H1x / self.dZ2x (the dW2 operands)."""
        L = self.L
        mb = self.mb if mb is None else int(mb)
        check(_lib.lib().satrl_ppo_rowpass_kx(L.H, mb, int(net), ptr(src), None if idx is None else ptr(idx),
                                              ptr(L.P), ptr(L.W2T), float(L.epsilon), float(L.entropy_coef),
                                              float(L.max_action), ptr(self.H1x), ptr(self.dZ2x), self.H1x.numel(),
                                              ptr(self.ptail), ptr(self.pw1), stream_ptr()), "satrl_ppo_rowpass_kx")

    def dw2_kx(self, mb, S, net=-1):
        """satrl_ppo_dw2_kx: the dW2 split-K slabs from the k-packed planes."""
        check(_lib.lib().satrl_ppo_dw2_kx(self.L.H, int(mb), int(net), int(S), ptr(self.H1x), ptr(self.dZ2x),
                                          self.H1x.numel(), ptr(self.p2), self.p2.numel(), stream_ptr()),
              "satrl_ppo_dw2_kx")

    def dw2_kx_w1(self, mb, S, net, mode, nsq):
        """satrl_ppo_dw2_kx_w1: dw2_kx with the reduce's W1 / tail regions
        (G, and their norm pairs with mode 3) in the same launch; returns the
        reduce mode bit that leaves it the W2 region (4), or 0 when the
        library has no such entry (an older development build: A/B only)."""
        lib = _lib.lib()
        if _lib.LIB_PATH != _lib._PRODUCT_LIB and not hasattr(lib, "satrl_ppo_dw2_kx_w1"):
            self.dw2_kx(mb, S, net)
            return 0
        check(lib.satrl_ppo_dw2_kx_w1(self.L.H, int(mb), int(net), int(S), ptr(self.H1x), ptr(self.dZ2x),
                                      self.H1x.numel(), ptr(self.p2), self.p2.numel(), int(mode), ptr(self.pw1),
                                      ptr(self.ptail), ptr(self.L.G), None if nsq is None else ptr(nsq), stream_ptr()),
              "satrl_ppo_dw2_kx_w1")
        return 4

    def rowpass_dw2(self, src, idx, mb=None, net=-1):
        """satrl_ppo_rowpass_dw2 (H = 64): the rowpass with each block's dW2
        partial written as split-K slab of p2 (no H1 / dZ2 stores)."""
        L = self.L
        mb = self.mb if mb is None else int(mb)
        check(_lib.lib().satrl_ppo_rowpass_dw2(L.H, mb, int(net), ptr(src), None if idx is None else ptr(idx),
                                               ptr(L.P), ptr(L.W2T), float(L.epsilon), float(L.entropy_coef),
                                               float(L.max_action), ptr(self.p2), self.p2.numel(), ptr(self.ptail),
                                               ptr(self.pw1), stream_ptr()), "satrl_ppo_rowpass_dw2")

    def rowpass_ratio(self, src, idx, ratio, mb=None, net=-1):
        """satrl_ppo_rowpass_ratio: satrl_ppo_rowpass that also writes the
        actor's probability ratio exp(logp - logp_old) per row into `ratio`."""
        L = self.L
        H = L.H
        mb = self.mb if mb is None else int(mb)
        n = 2 * mb * H
        _lib.require_cuda(ratio, torch.float32, (mb,), "ratio")
        check(_lib.lib().satrl_ppo_rowpass_ratio(H, mb, int(net), ptr(src), None if idx is None else ptr(idx),
                                                 ptr(L.P), ptr(L.W2T), float(L.epsilon), float(L.entropy_coef),
                                                 float(L.max_action), ptr(self.H1[:n]), ptr(self.dZ2[:n]),
                                                 ptr(self.ptail), ptr(self.pw1), ptr(ratio), stream_ptr()),
              "satrl_ppo_rowpass_ratio")
        return ratio

    def step_kernel_flops(self, mb=None):
        """Algorithmic FLOPs of the step's first launch: the rowpass, plus the
        dW2 product (2 H^2 per row and net) where it is fused in (H = 64)."""
        mb = self.mb if mb is None else int(mb)
        H = self.L.H
        return self.rowpass_flops(H, mb) + (2 * 2 * H * H * mb if self.fused_dw2 else 0)

    @staticmethod
    def rowpass_flops(H, mb):
        """Algorithmic FLOPs of one rowpass launch over both nets (DESIGN.md
        "Roofline"): per row and net fc1 forward + [dW1|db1] (2*18*H + H
        each), fc2 forward and dH1 (2*H*H each); output layers forward /
        backward (actor 3 outputs x 3 products, critic 1 x 3)."""
        per_row = 2 * (2 * (2 * 18 * H + H) + 2 * (2 * H * H)) + 2 * 3 * 3 * H + 2 * 1 * 3 * H
        return per_row * mb

    def max_splits(self, H):
        """Upper bound of splits(H, mb) over every mb (the p2 capacity)."""
        if self.fused_dw2:
            return self.nwg                  # row blocks of the longest minibatch at or below mb
        if self.kx_on:
            return max(self.S, 256 // 32)    # (dw2_kx: <= 256 / 32 tiles splits over both nets)
        return max(self.S, 256 // (2 * (H // 64) ** 2))

    def splits(self, H, mb):
        """split-K ways of the dW2 product for a minibatch of mb rows (both
        nets' count: a one-net chain of split mode uses the same)."""
        if self.fused_dw2:
            S = _lib.lib().satrl_ppo_row_blocks(int(H), int(mb))      # one slab per rowpass row block
            if S < 1:
                raise _lib.NativeError(f"satrl_ppo_row_blocks({H}, {mb}) failed")
            return S
        if self.kx(mb):
            S = _lib.lib().satrl_ppo_dw2_kx_splits(int(H), int(mb), -1)
            if S < 1:
                raise _lib.NativeError(f"satrl_ppo_dw2_kx_splits({H}, {mb}) failed")
            return S
        S = _lib.lib().satrl_ppo_dw2_splits(int(H), int(mb))
        if S < 1:
            raise _lib.NativeError(f"satrl_ppo_dw2_splits({H}, {mb}) failed")
        return S

    def _dw2(self, H1, dZ2, mb, S, net):
        """dW2 = dZ2^T @ H1 split-K S ways into the slabs p2 [2][S][H][H] (f32 rows)."""
        check(_lib.lib().satrl_ppo_dw2(self.L.H, mb, net, S, ptr(H1), ptr(dZ2), ptr(self.p2), self.p2.numel(),
                                       stream_ptr()), "satrl_ppo_dw2")

    def _net_step(self, src, idx, mb, net, events=None, skip_rowpass=False):
        """One minibatch step of one chain.  Bench-only knobs: `events` (a pair
        of torch.cuda.Event) recorded around the rowpass launch; skip_rowpass
        runs the rest of the chain on the last H1/dZ2/slabs (timing only)."""
        L = self.L
        H = L.H
        S = self.S if mb == self.mb else self.splits(H, mb)
        if S > self.p2_splits:
            raise _lib.NativeError(f"dW2 split count {S} exceeds the slab capacity {self.p2_splits}")
        lib, sp = _lib.lib(), stream_ptr()
        nsq = self.nsq[max(net, 0)]
        if events is not None:
            events[0].record()
        kx = self.kx(mb)
        if skip_rowpass:
            n = 2 * mb * H
            H1, dZ2 = self.H1[:n], self.dZ2[:n]
        elif kx:
            self.rowpass_kx(src, idx, mb, net)
            H1 = dZ2 = None
        elif self.fused_dw2:
            self.rowpass_dw2(src, idx, mb, net)
            H1 = dZ2 = None
        else:
            H1, dZ2 = self.rowpass(src, idx, mb, net)
        if events is not None:
            events[1].record()
        # H = 256: the reduce's W1 / tail regions ride in the dW2 launch
        # (satrl_ppo_dw2_kx_w1), the reduce sums the W2 region (mode bit 4)
        if L.pg is None:
            w2 = 0
            if kx:
                w2 = self.dw2_kx_w1(mb, S, net, 3, nsq)
            elif not self.fused_dw2:
                self._dw2(H1, dZ2, mb, S, net)
            check(lib.satrl_ppo_reduce(H, mb, net, S, 3 | w2, ptr(self.p2), self.p2.numel(), ptr(self.pw1),
                                       ptr(self.ptail), ptr(L.G), ptr(nsq), ptr(L.steps), sp), "satrl_ppo_reduce")
        else:
            w2 = 0
            if kx:
                w2 = self.dw2_kx_w1(mb, S, net, 1, None)
            elif not self.fused_dw2:
                self._dw2(H1, dZ2, mb, S, net)
            check(lib.satrl_ppo_reduce(H, mb, net, S, 1 | w2, ptr(self.p2), self.p2.numel(), ptr(self.pw1),
                                       ptr(self.ptail), ptr(L.G), None, None, sp), "satrl_ppo_reduce")
            # one bucket, both nets: SUM over the ranks, then G /= world and the norms in one launch
            if L.peer is not None and net < 0:
                L.peer.all_reduce_dp_(H, mb, L.G, nsq, L.steps)              # peer kernel, reduce_dp fused
            elif L.comm is not None:
                L.comm.all_reduce_sum_(L.G)                                   # RCCL on this stream (capturable)
            else:
                _dist.sum_inplace_(L.G, L.pg)                                 # c10d (gloo in the CPU tests)
            if L.peer is None or net >= 0:
                check(lib.satrl_ppo_reduce_dp(H, mb, net, _dist.world_size(L.pg), ptr(L.G), ptr(nsq), ptr(L.steps),
                                              sp), "satrl_ppo_reduce_dp")
        check(lib.satrl_ppo_adam(H, mb, net, ptr(nsq), ptr(L.steps), ptr(L.bct), L.bct.shape[0], ptr(L.lr),
                                 float(L.beta1), float(L.beta2), float(L.adam_eps), 0.5, int(bool(L.use_grad_clip)),
                                 ptr(L.G), ptr(L.P), ptr(L.M), ptr(L.V), ptr(L.W2T), sp), "satrl_ppo_adam")

    def _chains(self, fn):
        """fn(net) for the actor on the current stream and the critic on the
        side stream (fork/join), or fn(-1) once when not split."""
        if not self.split:
            fn(-1)
            return
        cur = torch.cuda.current_stream()
        self.side.wait_stream(cur)
        fn(0)
        with torch.cuda.stream(self.side):
            fn(1)
        cur.wait_stream(self.side)

    def step(self, src, idx, mb=None, events=None, skip_rowpass=False):
        mb = self.mb if mb is None else int(mb)
        if events is not None or skip_rowpass:
            self._net_step(src, idx, mb, -1, events, skip_rowpass)
            return
        self._chains(lambda net: self._net_step(src, idx, mb, net))

    def _group(self, src, ng):
        """ng minibatches whose indices are in self.idx[:ng]: one gather of
        their rows into self.stage, then ng steps per chain on contiguous rows."""
        mb = self.mb
        torch.index_select(src, 0, self.idx[:ng].view(-1), out=self.stage[:ng * mb])

        def chain(net):
            for k in range(ng):
                self._net_step(self.stage[k * mb:(k + 1) * mb], None, mb, net)
        self._chains(chain)

    def _group_dev(self, src):
        """One graph group: stage the rows of the next `group` minibatches of
        self.perm_buf (offset grp[0]), step them, advance grp."""
        mb, G = self.mb, self.group
        check(_lib.lib().satrl_ppo_stage(G * mb, ptr(src), ptr(self.perm_buf), ptr(self.grp), ptr(self.stage),
                                         stream_ptr()), "satrl_ppo_stage")

        def chain(net):
            for k in range(G):
                self._net_step(self.stage[k * mb:(k + 1) * mb], None, mb, net)
        self._chains(chain)
        check(_lib.lib().satrl_ppo_group_advance(ptr(self.grp), stream_ptr()), "satrl_ppo_group_advance")

    def _capture(self, src):
        if self.L.comm is not None:
            self.L.comm.warm(self.L.G)        # RCCL connects lazily: never inside the capture
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._group_dev(src)
        self._src_ptr = src.data_ptr()

    def run(self, src, perm):
        """All minibatches of one epoch (BatchSampler drop_last=False order)."""
        B = perm.numel()
        mb, G = self.mb, self.group
        nfull = B // mb
        graphable = self.use_graph and torch.cuda.is_available() and (self.L.pg is None or self.L.comm is not None
                                                                       or self.L.peer is not None)
        k = 0
        if graphable and nfull >= G:
            if self.perm_buf is None or self.perm_buf.numel() < B:
                self.perm_buf = torch.empty(B, dtype=torch.int64, device=perm.device)
                self.graph = None
            if perm.data_ptr() != self.perm_buf.data_ptr():
                self.perm_buf[:B].copy_(perm)
            if self.graph is None or self._src_ptr != src.data_ptr():
                self._capture(src)
            self.grp.zero_()
            comm, peer = self.L.comm, self.L.peer
            inflight = []
            for _ in range(nfull // G):
                self.graph.replay()
                if comm is not None or peer is not None:
                    # watchdog between replays: at most two replays queued ahead
                    # of the host.  RCCL: the oldest is waited for with the
                    # deadline while ncclCommGetAsyncError is polled
                    # (rccl.Comm.wait_event); peer: the oldest is polled against
                    # a host deadline, then the error word is read on a side
                    # stream (the queued replays keep running), so a lost rank
                    # stops the update there
                    ev = torch.cuda.Event()
                    ev.record()
                    inflight.append(ev)
                    if len(inflight) > 2:
                        if comm is not None:
                            comm.wait_event(inflight.pop(0), _dist.dp_timeout_s())
                        else:
                            peer.wait_event(inflight.pop(0))
            k = (nfull // G) * G
        while k < nfull:                      # the rest of the full minibatches, eagerly
            ng = min(G, nfull - k)
            self.idx[:ng].copy_(perm[k * mb:(k + ng) * mb].view(ng, mb))
            self._group(src, ng)
            k += ng
        if B % mb:
            tail = perm[nfull * mb:].contiguous()
            self.step(src, tail, mb=tail.numel())


def adam_bias_table(beta1=0.9, beta2=0.999):
    """{1 - beta1**k, sqrt(1 - beta2**k)} in python-float math, as
    torch.optim.Adam._single_tensor_adam computes them per step; rows up to
    the step where both are exactly 1.0."""
    rows = [(0.0, 0.0)]
    k = 1
    while True:
        b1 = 1 - beta1 ** k
        b2 = math.sqrt(1 - beta2 ** k)
        rows.append((b1, b2))
        if b1 == 1.0 and b2 == 1.0:
            break
        k += 1
    return torch.tensor(rows, dtype=torch.float64)


def _bind(module, name, view):
    """Make module.<name> a Parameter that aliases ``view`` (flat storage)."""
    module._parameters[name] = nn.Parameter(view, requires_grad=False)


class PPOLearner:
    """Actor/critic pair whose parameters, gradients and Adam moments live in
    flat device buffers (include/satrl_ppo.h layout); the nn.Module
    parameters are views into ``P`` so every forward pass (rollout, values,
    evaluate) reads the weights the fused update writes."""

    def __init__(self, args, agent_idx, device=None, pg=None, graph_group=16, use_graph=True):
        self.device = torch.device("cuda") if device is None else torch.device(device)
        self.args = args
        self.H = int(args.hidden_width)
        if not args.use_tanh:
            raise NotImplementedError("the fused update implements the tanh networks (use_tanh=True, CPPO_main.py:38)")
        self.max_action = float(args.max_action)
        self.batch_size = args.batch_size
        self.mini_batch_size = args.mini_batch_size
        self.max_train_steps = args.max_train_steps
        self.lr_a, self.lr_c = args.lr_a, args.lr_c
        self.gamma, self.lamda = args.gamma, args.lamda
        self.epsilon = args.epsilon
        self.K_epochs = args.K_epochs
        self.entropy_coef = args.entropy_coef
        self.use_grad_clip = args.use_grad_clip
        self.use_lr_decay = args.use_lr_decay
        self.use_adv_norm = args.use_adv_norm
        self.beta1, self.beta2 = 0.9, 0.999                  # torch.optim.Adam defaults
        self.adam_eps = 1e-5 if args.set_adam_eps else 1e-8  # ppo_continuous.py:161-166
        self.pg = pg
        # RCCL communicator for the in-graph gradient all-reduce (None without a
        # process group, or on gloo: the c10d all-reduce then runs eagerly)
        mode = getattr(args, "allreduce", "rccl")
        if mode not in ("rccl", "peer"):
            raise ValueError("allreduce must be 'rccl' or 'peer'")
        on_gpus = pg is not None and self.device.type == "cuda"
        self.comm = _rccl.for_group(pg, self.device) if on_gpus and mode == "rccl" else None
        self.peer = None
        if on_gpus and mode == "peer":
            from .peer import PeerComm
            self.peer = PeerComm(pg, ppo_layout(int(args.hidden_width))["total"], self.device, int(args.hidden_width))
        self.graph_group = graph_group
        self.use_graph = use_graph
        # CPU init with the reference's RNG consumption order (actor, then critic)
        actor = Actor_Gaussian(args, agent_idx)
        critic = Critic(args, agent_idx)
        self.off = ppo_layout(self.H)
        H, o = self.H, self.off
        f32 = dict(dtype=torch.float32, device=self.device)
        self.P = torch.zeros(o["total"], **f32)
        self.G = torch.zeros(o["total"], **f32)
        self.M = torch.zeros(o["total"], **f32)
        self.V = torch.zeros(o["total"], **f32)
        self.steps = torch.zeros(2, dtype=torch.float64, device=self.device)
        self.bct = adam_bias_table(self.beta1, self.beta2).to(self.device)
        self.lr = torch.tensor([float(self.lr_a), float(self.lr_c)], **f32)
        self.actor = actor.to(self.device)
        self.critic = critic.to(self.device)
        P = self.P
        self.W2v = P[o["W2"]:o["W2"] + 2 * H * H].view(2, H, H)
        # the fc2 operand image the rowpass reads (the f32 fc2.weight^T; satrl_ppo.h)
        self.W2T = torch.zeros(w2x_floats(H), **f32)
        self.GW2v = self.G[o["W2"]:o["W2"] + 2 * H * H].view(2, H, H)
        W1 = P[o["W1"]:o["W1"] + 2 * H * 20].view(2, H, 20)
        self.GW1v = self.G[o["W1"]:o["W1"] + 2 * H * 20].view(2, H, 20)
        b2 = P[o["b2"]:o["b2"] + 2 * H].view(2, H)
        views = {
            (self.actor.fc1, "weight"): W1[0, :, :18], (self.actor.fc1, "bias"): W1[0, :, 18],
            (self.critic.fc1, "weight"): W1[1, :, :18], (self.critic.fc1, "bias"): W1[1, :, 18],
            (self.actor.fc2, "weight"): self.W2v[0], (self.actor.fc2, "bias"): b2[0],
            (self.critic.fc2, "weight"): self.W2v[1], (self.critic.fc2, "bias"): b2[1],
            (self.actor.mean_layer, "weight"): P[o["W3a"]:o["W3a"] + 3 * H].view(3, H),
            (self.actor.mean_layer, "bias"): P[o["b3a"]:o["b3a"] + 3],
            (self.actor, "log_std"): P[o["ls"]:o["ls"] + 3].view(1, 3),
            (self.critic.fc3, "weight"): P[o["W3c"]:o["W3c"] + H].view(1, H),
            (self.critic.fc3, "bias"): P[o["b3c"]:o["b3c"] + 1],
        }
        with torch.no_grad():
            for (mod, name), view in views.items():
                view.copy_(getattr(mod, name).detach())
                _bind(mod, name, view)
        self._steppers = {}

    # -- lr ---------------------------------------------------------------------
    def lr_decay(self, total_steps):
        """ppo_continuous.py:244-250.  The reference's total_steps is an
        episode index below max_train_steps (its loop stops there,
        CPPO_main.py:110); the vectorised engine counts finished episodes over
        all envs and ranks, which can pass the budget inside an iteration, so
        the progress fraction is clamped to [0, 1] and lr never goes negative
        (identical to the reference wherever the reference runs)."""
        frac = min(max(float(total_steps) / self.max_train_steps, 0.0), 1.0)
        lr_a_now = self.lr_a * (1 - frac)
        lr_c_now = self.lr_c * (1 - frac)
        self.lr.copy_(torch.tensor([lr_a_now, lr_c_now], dtype=torch.float32))

    @property
    def lr_now(self):
        v = self.lr.cpu().tolist()
        return v[0], v[1]

    def param_groups(self):
        """(actor params, critic params) as tensors, reference order."""
        return list(self.actor.parameters()), list(self.critic.parameters())

    def flat_views(self, buf):
        """{"actor.fc1.weight": view, ...} of a flat buffer (P, G, M or V)."""
        H, o = self.H, self.off
        W1 = buf[o["W1"]:o["W1"] + 2 * H * 20].view(2, H, 20)
        W2 = buf[o["W2"]:o["W2"] + 2 * H * H].view(2, H, H)
        b2 = buf[o["b2"]:o["b2"] + 2 * H].view(2, H)
        return {"actor.fc1.weight": W1[0, :, :18], "actor.fc1.bias": W1[0, :, 18],
                "actor.fc2.weight": W2[0], "actor.fc2.bias": b2[0],
                "actor.mean_layer.weight": buf[o["W3a"]:o["W3a"] + 3 * H].view(3, H),
                "actor.mean_layer.bias": buf[o["b3a"]:o["b3a"] + 3],
                "actor.log_std": buf[o["ls"]:o["ls"] + 3].view(1, 3),
                "critic.fc1.weight": W1[1, :, :18], "critic.fc1.bias": W1[1, :, 18],
                "critic.fc2.weight": W2[1], "critic.fc2.bias": b2[1],
                "critic.fc3.weight": buf[o["W3c"]:o["W3c"] + H].view(1, H),
                "critic.fc3.bias": buf[o["b3c"]:o["b3c"] + 1]}

    # -- update -----------------------------------------------------------------
    def sync_w2t(self):
        """Refresh the fc2 operand image from P (Adam keeps it current during an
        update; this covers loads / external writes between updates)."""
        if self.device.type == "cuda":
            check(_lib.lib().satrl_ppo_w2x_sync(self.H, -1, ptr(self.P), ptr(self.W2T), stream_ptr()),
                  "satrl_ppo_w2x_sync")
        else:
            self.W2T.copy_(w2x_image(self.P[:2 * self.H * self.H], self.H))

    def w2t_f32(self):
        """fc2.weight^T per net [2, H, H] f32 from the operand image."""
        return w2x_decode(self.W2T, self.H)

    def stepper(self, mb):
        if mb not in self._steppers:
            self._steppers[mb] = FusedMinibatch(self, mb, self.graph_group, use_graph=self.use_graph)
        return self._steppers[mb]

    def normalize_adv(self, adv):
        """ppo_continuous.py:209-210 (unbiased std); global over the process group."""
        if not self.use_adv_norm:
            return adv
        if self.pg is None:
            return (adv - adv.mean()) / (adv.std() + 1e-5)
        cnt = torch.tensor([float(adv.numel())], dtype=torch.float64, device=adv.device)
        mean, std = _dist.global_mean_std(torch.cat([moments(adv), cnt]), self.pg)
        return (adv - mean.float()) / (std.float() + 1e-5)

    def update_packed(self, src, total_steps, perms=None, generator=None):
        """K epochs of minibatch steps over the packed table src [B, 32]
        (adv already normalised), then lr decay (ppo_continuous.py:212-242)."""
        B = src.shape[0]
        self.sync_w2t()
        st = self.stepper(min(self.mini_batch_size, B))
        for ep in range(self.K_epochs):
            if perms is None:
                perm = torch.randperm(B, device=self.device, generator=generator)
            else:
                perm = perms(ep) if callable(perms) else perms[ep]     # a callable draws each epoch's order lazily
            st.run(src, perm)
        if self.peer is not None:
            self.peer.check()                # a peer's value never arrived: the update is invalid
        if uses_column_split(self.H, self.mini_batch_size, B):
            rowpass_exchange_check()         # (minibatches / tails <= 1024 rows; bounded by the DP deadline)
        if self.use_lr_decay:
            self.lr_decay(total_steps)

    @staticmethod
    def pack(s, a, logp, adv, vt, out=None):
        B = s.shape[0]
        out = torch.empty((B, 32), dtype=torch.float32, device=s.device) if out is None else out
        out[:, 0:18] = s
        out[:, 18:21] = a
        out[:, 21:24] = logp
        out[:, 24] = adv.reshape(-1)
        out[:, 25] = vt.reshape(-1)
        out[:, 26:] = 0
        return out


class HostLearner:
    """The N = 1 drop-in's agent on host cores (device="cpu"; BASELINE.json
    configs[0]: CPPO_main.py on CPU, no GPU).  The networks are the same
    nn.Modules, stepped by torch's CPU autograd, clip_grad_norm_ and Adam in
    the order of ppo_continuous.py:212-239 (actor step, then critic step, per
    minibatch); the vectorised engine never uses it (its update is the HIP
    minibatch step of PPOLearner)."""

    def __init__(self, args, agent_idx):
        self.device = torch.device("cpu")
        self.actor = Actor_Gaussian(args, agent_idx)
        self.critic = Critic(args, agent_idx)
        self.lr_a, self.lr_c = args.lr_a, args.lr_c
        self.max_train_steps = args.max_train_steps
        self.K_epochs, self.epsilon, self.entropy_coef = args.K_epochs, args.epsilon, args.entropy_coef
        self.use_grad_clip, self.use_lr_decay, self.use_adv_norm = (args.use_grad_clip, args.use_lr_decay,
                                                                   args.use_adv_norm)
        kw = {"eps": 1e-5} if args.set_adam_eps else {}                  # ppo_continuous.py:161-166
        self.opts = (torch.optim.Adam(self.actor.parameters(), lr=self.lr_a, **kw),
                     torch.optim.Adam(self.critic.parameters(), lr=self.lr_c, **kw))

    def normalize_adv(self, adv):
        return (adv - adv.mean()) / (adv.std() + 1e-5) if self.use_adv_norm else adv

    def lr_decay(self, total_steps):
        frac = min(max(float(total_steps) / self.max_train_steps, 0.0), 1.0)    # as PPOLearner.lr_decay
        for opt, lr in zip(self.opts, (self.lr_a, self.lr_c)):
            for g in opt.param_groups:
                g["lr"] = lr * (1 - frac)

    @property
    def lr_now(self):
        return tuple(opt.param_groups[0]["lr"] for opt in self.opts)

    def _minibatch(self, rows):
        # contiguous column blocks, as the reference's s[index], a[index] ... are
        s, a, lp_old, adv, vt = (rows[:, lo:hi].contiguous() for lo, hi in ((0, 18), (18, 21), (21, 24), (24, 25),
                                                                             (25, 26)))
        dist = self.actor.get_dist(s)
        ent = dist.entropy().sum(1, keepdim=True)
        ratio = torch.exp(dist.log_prob(a).sum(1, keepdim=True) - lp_old.sum(1, keepdim=True))
        loss = -torch.min(ratio * adv, torch.clamp(ratio, 1 - self.epsilon, 1 + self.epsilon) * adv)
        losses = ((loss - self.entropy_coef * ent).mean(), lambda: F.mse_loss(vt, self.critic(s)))
        for k, (net, opt) in enumerate(zip((self.actor, self.critic), self.opts)):
            opt.zero_grad()
            (losses[0] if k == 0 else losses[1]()).backward()
            if self.use_grad_clip:
                torch.nn.utils.clip_grad_norm_(net.parameters(), 0.5)
            opt.step()

    def update_packed(self, src, total_steps, perms):
        """K epochs over the packed rows [B, 32] in the given minibatch orders."""
        mb = self.mini_batch_size
        for ep in range(self.K_epochs):
            perm = perms[ep]
            for k in range(0, perm.numel(), mb):
                self._minibatch(src[perm[k:k + mb]])
        if self.use_lr_decay:
            self.lr_decay(total_steps)


def _gae_host(r, vs, vs_, dw, done, gamma, lamda):
    """ppo_continuous.py:198-208 on host arrays: f32 deltas, then the reverse
    scan with numpy-scalar arithmetic (f32, python floats weak) as the
    reference's loop runs it."""
    deltas = (r + gamma * (1.0 - dw) * vs_ - vs).reshape(-1).numpy()
    d = done.reshape(-1).numpy()
    adv = np.empty_like(deltas)
    g = 0
    for t in range(len(deltas) - 1, -1, -1):
        g = deltas[t] + gamma * lamda * g * (1.0 - d[t])
        adv[t] = g
    adv = torch.from_numpy(adv)
    return adv, adv + vs.reshape(-1)


class PPO_continuous:  # noqa: N801
    """Drop-in for ppo_continuous.PPO_continuous (ppo_continuous.py:136-258).

    Networks and optimizer live on the GPU.  ``choose_action`` draws its
    noise from torch's global CPU generator exactly as the reference's
    ``Normal.sample()`` does, and ``update`` draws its minibatch permutations
    from the same generator (BatchSampler(SubsetRandomSampler), drop_last
    False), so seeding and indexing match the reference bit for bit.
    """

    def __init__(self, args, agent_idx, device=None):
        if args.policy_dist != "Gaussian":
            raise NotImplementedError("only the Gaussian policy (CPPO_main.py:17 default) is on the hot path")
        self.policy_dist = args.policy_dist
        dev = device if device is not None else getattr(args, "device", None)
        if dev is not None and torch.device(dev).type == "cpu":
            self.L = HostLearner(args, agent_idx)          # device="cpu" only when asked (configs[0])
            self.L.mini_batch_size = args.mini_batch_size
        else:
            self.L = PPOLearner(args, agent_idx, device=device, graph_group=4)
        self.actor, self.critic = self.L.actor, self.L.critic
        self.max_action = args.max_action
        self.batch_size = args.batch_size
        self.mini_batch_size = args.mini_batch_size
        self.K_epochs = args.K_epochs
        self.gamma, self.lamda = args.gamma, args.lamda

    def _obs(self, s):
        return torch.as_tensor(np.asarray(s), dtype=torch.float32).reshape(1, -1).to(self.L.device)

    def evaluate(self, s):
        """ppo_continuous.py:168-174 (mean action)."""
        with torch.no_grad():
            return self.actor(self._obs(s)).cpu().numpy().flatten()

    def choose_action(self, s):
        """ppo_continuous.py:176-189."""
        with torch.no_grad():
            mean = self.actor(self._obs(s)).cpu()
            std = torch.exp(self.actor.log_std.detach().cpu().expand_as(mean))
            dist = torch.distributions.Normal(mean, std)
            a = dist.sample()
            a = torch.clamp(a, -self.max_action, self.max_action)
            a_logprob = dist.log_prob(a)
        return a.numpy().flatten(), a_logprob.numpy().flatten()

    def update(self, replay_buffer, total_steps):
        """ppo_continuous.py:191-242 on a flat ReplayBuffer."""
        from torch.utils.data.sampler import BatchSampler, SubsetRandomSampler
        dev = self.L.device
        s, a, a_logprob, r, s_, dw, done = [t.to(dev) for t in replay_buffer.numpy_to_tensor()]
        B = s.shape[0]
        with torch.no_grad():
            vs = self.critic(s)
            vs_ = self.critic(s_)
            gae_fn = _gae_host if isinstance(self.L, HostLearner) else _gae_explicit
            adv, v_target = gae_fn(r.reshape(-1), vs.reshape(-1), vs_.reshape(-1), dw.reshape(-1),
                                   done.reshape(-1), self.gamma, self.lamda)
            adv = adv.reshape(-1, 1)
            v_target = v_target.reshape(-1, 1)
            adv = self.L.normalize_adv(adv)
        src = PPOLearner.pack(s, a, a_logprob, adv, v_target)
        perms = []
        for _ in range(self.K_epochs):
            idx = [i for batch in BatchSampler(SubsetRandomSampler(range(B)), self.mini_batch_size, False)
                   for i in batch]
            perms.append(torch.tensor(idx, dtype=torch.int64, device=dev))
        self.L.update_packed(src, total_steps, perms=perms)

    def lr_decay(self, total_steps):
        self.L.lr_decay(total_steps)

    def save_checkpoint(self):
        self.actor.save_checkpoint()
        self.critic.save_checkpoint()

    def load_checkpoint(self):
        self.actor.load_checkpoint()
        self.critic.load_checkpoint()


def _gae_explicit(r, vs, vs_, dw, done, gamma, lamda):
    """General flat-buffer GAE with separate V(s') (dw != done boundaries):
    runs the HIP scan on a one-column buffer whose deltas already carry V(s')."""
    B = r.shape[0]
    # delta_t = r + g(1-dw)V(s') - V(s): feed r' = r + g(1-dw)V(s') - V(s) + V(s) ... keep the
    # reference order by computing deltas here, then scanning with V == 0.
    deltas = r + gamma * (1.0 - dw) * vs_ - vs
    zeros = torch.zeros(B + 1, 1, dtype=torch.float32, device=r.device)
    adv, _ = gae(deltas.reshape(B, 1).contiguous(), done.reshape(B, 1).to(torch.uint8).contiguous(), zeros,
                 gamma, lamda)
    adv = adv.reshape(-1)
    return adv, adv + vs
