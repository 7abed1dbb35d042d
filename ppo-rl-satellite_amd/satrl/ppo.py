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

import math
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
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
        torch.save(self.state_dict(), self.chkpt_file)

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
        torch.save(self.state_dict(), self.chkpt_file)

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


def moments(x, out=None):
    out = torch.zeros(2, dtype=torch.float64, device=x.device) if out is None else out
    x = x.reshape(-1)
    check(_lib.lib().satrl_moments(x.numel(), ptr(x), ptr(out), stream_ptr()), "satrl_moments")
    return out


# ---------------------------------------------------------------------------
# minibatch step (ppo_continuous.py:213-239)
# ---------------------------------------------------------------------------
class MinibatchStepper:
    """Actor + critic clipped-surrogate / MSE step on index batches.

    The step for a fixed minibatch size is captured once into a hipGraph
    holding ``group`` consecutive minibatches; each replay consumes one
    [group, mb] block of a device permutation.  ``src`` is the packed
    transition table [B, 32] f32: s(18) a(3) logp(3) adv(1) v_target(1) pad.
    With a process group, gradients of both nets are averaged with one
    bucketed all-reduce per minibatch (eager, between two captured halves).
    """

    S, A, LP, ADV, VT = slice(0, 18), slice(18, 21), slice(21, 24), slice(24, 25), slice(25, 26)

    def __init__(self, learner, mb, group, pg=None, use_graph=True):
        self.L = learner
        self.mb = mb
        self.group = group
        self.pg = pg
        self.use_graph = use_graph and torch.cuda.is_available()
        dev = learner.device
        self.idx = torch.zeros((group, mb), dtype=torch.int64, device=dev)
        self.graph = None
        self.graph_b = None
        self._src_ptr = None

    # one minibatch: ppo_continuous.py:216-239, actor first then critic
    def _actor_loss(self, rows):
        L = self.L
        s, a, lp_old, adv = rows[:, self.S], rows[:, self.A], rows[:, self.LP], rows[:, self.ADV]
        mean = L.actor(s)
        log_std = L.actor.log_std.expand_as(mean)
        std = torch.exp(log_std)
        var = std ** 2
        log_scale = std.log()
        logp = -((a - mean) ** 2) / (2 * var) - log_scale - LOG_SQRT_2PI        # Normal.log_prob
        ent = (ENT_CONST + torch.log(std)).sum(1, keepdim=True)                 # Normal.entropy().sum(1)
        ratios = torch.exp(logp.sum(1, keepdim=True) - lp_old.sum(1, keepdim=True))
        surr1 = ratios * adv
        surr2 = torch.clamp(ratios, 1 - L.epsilon, 1 + L.epsilon) * adv
        return (-torch.min(surr1, surr2) - L.entropy_coef * ent).mean()

    def _critic_loss(self, rows):
        return F.mse_loss(rows[:, self.VT], self.L.critic(rows[:, self.S]))

    def _fwd_bwd(self, src, idx):
        L = self.L
        rows = src.index_select(0, idx)
        L.opt_a.zero_grad(set_to_none=False)
        self._actor_loss(rows).backward()
        L.opt_c.zero_grad(set_to_none=False)
        self._critic_loss(rows).backward()

    def _apply(self):
        L = self.L
        if L.use_grad_clip:
            torch.nn.utils.clip_grad_norm_(L.actor_params, 0.5)
        L.opt_a.step()
        if L.use_grad_clip:
            torch.nn.utils.clip_grad_norm_(L.critic_params, 0.5)
        L.opt_c.step()

    def _allreduce(self):
        import torch.distributed as dist
        L = self.L
        grads = [p.grad for p in L.actor_params + L.critic_params]
        flat = torch._utils._flatten_dense_tensors(grads)
        dist.all_reduce(flat, group=self.pg)
        flat.div_(dist.get_world_size(self.pg))
        for g, f in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
            g.copy_(f)

    def _eager_group(self, src, ng):
        for k in range(ng):
            self._fwd_bwd(src, self.idx[k])
            if self.pg is not None:
                self._allreduce()
            self._apply()

    def _capture(self, src):
        # warm up on a side stream (allocates grads / optimizer state), then capture
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._fwd_bwd(src, self.idx[0])
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for k in range(self.group):
                self._fwd_bwd(src, self.idx[k])
                self._apply()
        self._src_ptr = src.data_ptr()

    def run(self, src, perm):
        """Run all minibatches of one epoch; perm int64 [B] on device."""
        B = perm.numel()
        mb, G = self.mb, self.group
        nfull = B // mb
        k = 0
        graphable = self.use_graph and self.pg is None
        if graphable and (self.graph is None or self._src_ptr != src.data_ptr()):
            # optimizer state must exist before capture: one eager warm step on a
            # zero-lr copy is not needed -- Adam(capturable) allocates lazily, so
            # the first group runs eagerly.
            if not self.L._opt_ready:
                ng = min(G, nfull)
                self.idx[:ng].copy_(perm[: ng * mb].view(ng, mb))
                self._eager_group(src, ng)
                self.L._opt_ready = True
                k = ng
            if nfull - k >= G:
                self._capture(src)
        while k < nfull:
            ng = min(G, nfull - k)
            self.idx[:ng].copy_(perm[k * mb:(k + ng) * mb].view(ng, mb))
            if graphable and ng == G and self.graph is not None:
                self.graph.replay()
            else:
                self._eager_group(src, ng)
            k += ng
        if B % mb:                                     # drop_last=False tail
            tail = perm[nfull * mb:]
            self._fwd_bwd(src, tail)
            if self.pg is not None:
                self._allreduce()
            self._apply()


class PPOLearner:
    """Actor/critic pair + optimizers + batched update (device resident)."""

    def __init__(self, args, agent_idx, device=None, pg=None, graph_group=16, use_graph=True):
        self.device = torch.device("cuda") if device is None else torch.device(device)
        self.args = args
        self.max_action = args.max_action
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
        # CPU init with the reference's RNG consumption order (actor, then critic)
        actor = Actor_Gaussian(args, agent_idx)
        critic = Critic(args, agent_idx)
        self.actor = actor.to(self.device)
        self.critic = critic.to(self.device)
        self.actor_params = list(self.actor.parameters())
        self.critic_params = list(self.critic.parameters())
        eps = 1e-5 if args.set_adam_eps else 1e-8
        self._lr_a_t = torch.tensor(float(self.lr_a), device=self.device)
        self._lr_c_t = torch.tensor(float(self.lr_c), device=self.device)
        self.opt_a = torch.optim.Adam(self.actor_params, lr=self._lr_a_t, eps=eps, capturable=True, foreach=True)
        self.opt_c = torch.optim.Adam(self.critic_params, lr=self._lr_c_t, eps=eps, capturable=True, foreach=True)
        self._opt_ready = False
        self.pg = pg
        self.graph_group = graph_group
        self.use_graph = use_graph
        self._steppers = {}

    # -- lr ---------------------------------------------------------------------
    def lr_decay(self, total_steps):
        """ppo_continuous.py:244-250."""
        lr_a_now = self.lr_a * (1 - total_steps / self.max_train_steps)
        lr_c_now = self.lr_c * (1 - total_steps / self.max_train_steps)
        self._lr_a_t.fill_(lr_a_now)
        self._lr_c_t.fill_(lr_c_now)
        for p in self.opt_a.param_groups:
            p["lr"] = self._lr_a_t
        for p in self.opt_c.param_groups:
            p["lr"] = self._lr_c_t

    @property
    def lr_now(self):
        return float(self._lr_a_t.item()), float(self._lr_c_t.item())

    # -- update -----------------------------------------------------------------
    def stepper(self, mb):
        if mb not in self._steppers:
            self._steppers[mb] = MinibatchStepper(self, mb, self.graph_group, pg=self.pg, use_graph=self.use_graph)
        return self._steppers[mb]

    def normalize_adv(self, adv):
        """ppo_continuous.py:209-210 (unbiased std); global over the process group."""
        if not self.use_adv_norm:
            return adv
        n_local = adv.numel()
        if self.pg is None:
            return (adv - adv.mean()) / (adv.std() + 1e-5)
        import torch.distributed as dist
        m = moments(adv)
        cnt = torch.tensor([float(n_local)], dtype=torch.float64, device=adv.device)
        buf = torch.cat([m, cnt])
        dist.all_reduce(buf, group=self.pg)
        s, s2, n = buf[0], buf[1], buf[2]
        mean = s / n
        var = (s2 - n * mean * mean) / (n - 1)
        return (adv - mean.float()) / (var.clamp_min(0).sqrt().float() + 1e-5)

    def update_packed(self, src, total_steps, perms=None, generator=None):
        """K epochs of minibatch steps over the packed table src [B, 32]
        (adv already normalised), then lr decay (ppo_continuous.py:212-242)."""
        B = src.shape[0]
        st = self.stepper(self.mini_batch_size)
        for ep in range(self.K_epochs):
            if perms is not None:
                perm = perms[ep]
            else:
                perm = torch.randperm(B, device=self.device, generator=generator)
            st.run(src, perm)
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
        self.L = PPOLearner(args, agent_idx, device=device, graph_group=4)
        self.actor, self.critic = self.L.actor, self.L.critic
        self.max_action = args.max_action
        self.batch_size = args.batch_size
        self.mini_batch_size = args.mini_batch_size
        self.K_epochs = args.K_epochs
        self.gamma, self.lamda = args.gamma, args.lamda

    @property
    def optimizer_actor(self):
        return self.L.opt_a

    @property
    def optimizer_critic(self):
        return self.L.opt_c

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
            adv, v_target = _gae_explicit(r.reshape(-1), vs.reshape(-1), vs_.reshape(-1), dw.reshape(-1),
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
