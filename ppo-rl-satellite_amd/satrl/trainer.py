"""Training loops.

* ``args_param`` -- CPPO_main.py:13-65 config surface (every reference
  keyword, same defaults) plus the engine's keywords (num_envs, horizon,
  seed, rollout_graph_chunk, update_graph_group).
* ``train_pursuer_network`` / ``train_evader_network`` / ``test_network`` --
  CPPO_main.py:94-282 semantics over the drop-in N=1 classes.
* ``VecTrainer`` -- the vectorised engine: N envs x T steps per iteration,
  collected by hipGraph-captured chunks of [actor fwd -> HIP sample (x2
  agents) -> HIP env step], then critic values, HIP GAE scan, global
  advantage normalisation, and the graph-captured minibatch update.
  One process per GPU; with a process group the envs are sharded by global
  env id (Philox noise keyed by it, so rollouts do not depend on sharding)
  and gradients are averaged with RCCL.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from . import dist as _dist
from .buffer import ReplayBuffer, RolloutBuffer
from .env import VecSatellites
from .ppo import PPO_continuous, PPOLearner, gae, gaussian_sample, policy_act, policy_value


class args_param:  # noqa: N801
    """CPPO_main.py:13-65 (same keywords and defaults) + engine keywords."""

    def __init__(self, max_train_steps=int(3e6), evaluate_freq=5e3, save_freq=20, policy_dist="Gaussian",
                 batch_size=2048, mini_batch_size=64, hidden_width=256, hidden_width2=128, lr_a=0.0002, lr_c=0.0002,
                 gamma=0.99, lamda=0.95, epsilon=0.1, K_epochs=10, max_episode_steps=1000, use_adv_norm=True,
                 use_state_norm=True, use_reward_norm=False, use_reward_scaling=True, entropy_coef=0.01,
                 use_lr_decay=True, use_grad_clip=True, use_orthogonal_init=True, set_adam_eps=True, use_tanh=True,
                 chkpt_dir="/mnt/datab/home/yuanwenzheng/PICTURE1",
                 num_envs=1, horizon=None, seed=0, rollout_graph_chunk=64, update_graph_group=64, device=None,
                 surrogate=False, dp_minibatch="global", minibatch_sampler=None, allreduce="rccl"):
        self.max_train_steps = max_train_steps
        self.evaluate_freq = evaluate_freq
        self.save_freq = save_freq
        self.policy_dist = policy_dist
        self.batch_size = batch_size
        self.mini_batch_size = mini_batch_size
        self.hidden_width = hidden_width
        self.hidden_width2 = hidden_width2
        self.lr_a = lr_a
        self.lr_c = lr_c
        self.gamma = gamma
        self.lamda = lamda
        self.epsilon = epsilon
        self.K_epochs = K_epochs
        self.use_adv_norm = use_adv_norm
        self.use_state_norm = use_state_norm
        self.use_reward_norm = use_reward_norm
        self.use_reward_scaling = use_reward_scaling
        self.entropy_coef = entropy_coef
        self.use_lr_decay = use_lr_decay
        self.use_grad_clip = use_grad_clip
        self.use_orthogonal_init = use_orthogonal_init
        self.set_adam_eps = set_adam_eps
        self.use_tanh = use_tanh
        self.max_episode_steps = max_episode_steps
        self.chkpt_dir = chkpt_dir
        # engine
        self.num_envs = num_envs
        self.horizon = horizon if horizon is not None else max(1, batch_size // max(1, num_envs))
        self.seed = seed
        self.rollout_graph_chunk = rollout_graph_chunk
        self.update_graph_group = update_graph_group
        self.device = device
        # config 5: evaluate the ImprovedNN surrogate (bf16) on every env step into
        # VecTrainer.ellipse_params (environment.py:158); True = the net trained on the
        # reference's golden pairs (satrl/data/improvednn_trained.npz, with its scalers);
        # a path or state_dict loads other weights
        self.surrogate = surrogate
        # data parallelism: "global" -- mini_batch_size is the
        # GLOBAL minibatch, each of W ranks steps mini_batch_size / W of its
        # rows per Adam step (the reference's minibatch semantics,
        # ppo_continuous.py:213); "per_gpu" -- every rank steps
        # mini_batch_size local rows (global minibatch mini_batch_size * W).
        self.dp_minibatch = dp_minibatch
        # minibatch index sampler of the vectorised engine: "uniform" =
        # BatchSampler(SubsetRandomSampler(range(B))) over the local table
        # (the reference's distribution); "stratified" = every minibatch holds
        # mini_batch_size / 8 rows of each of 8 fixed global env blocks, drawn
        # by per-block generators, so W = 1, 2, 4, 8 ranks draw the same
        # global minibatches (None: uniform on one process, stratified under
        # "global" data parallelism)
        self.minibatch_sampler = minibatch_sampler
        # the per-minibatch gradient all-reduce under data parallelism on GPUs:
        # "rccl" (ncclAllReduce + reduce_dp, in the update's graphs) or "peer"
        # (satrl_ppo_allreduce_peer: a two-shot reduce-scatter + all-gather
        # over IPC-mapped buffers, fused with reduce_dp; satrl/peer.py)
        self.allreduce = allreduce
        # set by the train_* functions from the env (CPPO_main.py:99-101)
        self.state_dim = 18
        self.action_dim = 3
        self.max_action = 1.6

    def print_information(self):
        for k, v in vars(self).items():
            print(f"{k}: {v}")


# ---------------------------------------------------------------------------
# reference loops (CPPO_main.py:94-282) on the drop-in N=1 classes
# ---------------------------------------------------------------------------
def _setup(args, env, d_capture):
    env.d_capture = d_capture                               # CPPO_main.py:98
    args.state_dim = env.observation_space.shape[0]
    args.action_dim = env.action_space.shape[0]
    args.max_action = float(env.action_space[0][1])


def _episode_loop(args, env, agents, learner, flag, stored_agent, update_agent, max_episodes, on_done=None):
    replay_buffer = ReplayBuffer(args)
    rewards, mean_rewards = [], []
    pursuer_agent, evader_agent = agents
    for epsiode in range(max_episodes):
        epsiode_reward = 0.0
        epsiode_count = 0
        s = env.reset(flag)
        while True:
            epsiode_count += 1
            pa, plp = pursuer_agent.choose_action(s)
            ea, elp = evader_agent.choose_action(s)
            s_, r, done = env.step(pa, ea, epsiode_count)
            epsiode_reward += r
            dw = bool(done or epsiode_count >= args.max_episode_steps)
            if stored_agent == "pursuer":
                replay_buffer.store(s, pa, plp, r, s_, dw, done)
            else:
                replay_buffer.store(s, ea, elp, r, s_, dw, done)
            s = s_
            if replay_buffer.count == args.batch_size:
                update_agent.update(replay_buffer, epsiode)
                replay_buffer.count = 0
            if done:
                rewards.append(epsiode_reward)
                mean_rewards.append(float(np.mean(rewards)))
                if on_done:
                    on_done(epsiode, epsiode_reward, mean_rewards[-1])
                break
    return rewards, mean_rewards


def train_pursuer_network(args, env, show_picture=False, pre_train=False, d_capture=0, max_episodes=None):
    """CPPO_main.py:94-161."""
    _setup(args, env, d_capture)
    pursuer_agent = PPO_continuous(args, "pursuer")
    evader_agent = PPO_continuous(args, "evader")
    if pre_train:
        pursuer_agent.load_checkpoint()
    n = args.max_train_steps if max_episodes is None else max_episodes
    rewards, means = _episode_loop(args, env, (pursuer_agent, evader_agent), pursuer_agent, 0, "pursuer",
                                   pursuer_agent, n)
    pursuer_agent.save_checkpoint()
    return pursuer_agent


def train_evader_network(args, env, show_picture=False, pre_train=False, d_capture=0, max_episodes=None,
                         fix_update_agent=False):
    """CPPO_main.py:163-230.  The reference updates ``pursuer_agent`` with the
    evader's transitions (CPPO_main.py:215); that is reproduced unless
    ``fix_update_agent`` is set."""
    _setup(args, env, d_capture)
    pursuer_agent = PPO_continuous(args, "pursuer")
    evader_agent = PPO_continuous(args, "evader")
    if pre_train:
        evader_agent.load_checkpoint()
    n = args.max_train_steps if max_episodes is None else max_episodes
    upd = evader_agent if fix_update_agent else pursuer_agent
    _episode_loop(args, env, (pursuer_agent, evader_agent), upd, 1, "evader", upd, n)
    evader_agent.save_checkpoint()
    return evader_agent


def test_network(args, env, show_pictures=False, d_capture=0):
    """CPPO_main.py:233-282; returns the episode return (the reference prints it)."""
    _setup(args, env, d_capture)
    pursuer_agent = PPO_continuous(args, "pursuer")
    evader_agent = PPO_continuous(args, "evader")
    pursuer_agent.load_checkpoint()
    epsiode_reward = 0.0
    epsiode_count = 0
    s = env.reset(0)
    while True:
        epsiode_count += 1
        pa, _ = pursuer_agent.choose_action(s)
        ea, _ = evader_agent.choose_action(s)
        s_, r, done = env.step(pa, ea, epsiode_count)
        epsiode_reward += r
        s = s_
        if done:
            print("当前测试得分为{}".format(epsiode_reward))
            return epsiode_reward


def train_elliptical_network(args, env, epsiodes=200, d_capture=0):
    """CPPO_main.py:284-322: Flag-2 episodes with the trained pursuer and an
    untrained evader acting; each env step fits the reachable-domain
    ellipse (GPU grid + fit kernels) and trains the env's ImprovedNN.  Note
    the reference never resets epsiode_count between episodes (:287, :301),
    so every episode after the first ends at its first step's timeout test."""
    env.d_capture = d_capture
    args.state_dim = env.observation_space.shape[0]
    args.action_dim = env.action_space.shape[0]
    args.max_action = float(env.action_space[0][1])
    pursuer_agent = PPO_continuous(args, "pursuer")
    evader_agent = PPO_continuous(args, "evader")
    pursuer_agent.load_checkpoint()
    epsiode_count = 0
    for _ in range(epsiodes):
        s = env.reset(2)
        while True:
            epsiode_count += 1
            pa, _ = pursuer_agent.choose_action(s)
            ea, _ = evader_agent.choose_action(s)
            if args.policy_dist == "Beta":
                pa = 2 * (pa - 0.5) * args.max_action
                ea = 2 * (ea - 0.5) * args.max_action
            s_, r, done = env.step(pa, ea, epsiode_count)
            s = s_
            if done:
                break


# ---------------------------------------------------------------------------
# vectorised engine
# ---------------------------------------------------------------------------
def stratified_epoch_perm(T, n_local, world, rank, global_mb, gens, strata=8, device=None):
    """One epoch's minibatch order for rank `rank` of `world`.

    The global table is [T, n_local * world] (row t * N_glob + global env),
    cut into `strata` blocks of consecutive global envs; rank r owns blocks
    [r * strata / world, (r + 1) * strata / world).  Block s draws its own
    permutation of its T * N_glob / strata rows from gens[s]; global
    minibatch k is the concatenation over blocks of their k-th chunk of
    global_mb / strata rows (the tail: the leftover rows of every block).  A
    rank returns its blocks' share in LOCAL rows (t * n_local + local env),
    minibatch-major, so every rank steps global_mb / world rows of each
    global minibatch and W = 1, 2, 4, 8 draw the same global minibatches."""
    Ns = n_local * world // strata
    Bs = T * Ns
    c = global_mb // strata
    nfull = Bs // c
    full, tail = [], []
    for s_ in range(rank * (strata // world), (rank + 1) * (strata // world)):
        q = torch.randperm(Bs, device=device, generator=gens[s_])
        t, e = q // Ns, q % Ns + (s_ * Ns - rank * n_local)
        loc = t * n_local + e
        full.append(loc[:nfull * c].view(nfull, c))
        tail.append(loc[nfull * c:])
    return torch.cat([torch.cat(full, 1).reshape(-1)] + tail)


class VecTrainer:
    """N envs x horizon T per iteration on one GPU (one process per GPU)."""

    def __init__(self, args, flag=0, d_capture=15000.0, device=None, pg=None, env_offset=0, use_graphs=True):
        self.args = args
        self.flag = int(flag)
        self.pg = pg
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.N = int(args.num_envs)
        self.T = int(args.horizon)
        self.env_offset = int(env_offset)
        self.seed = int(args.seed)
        args.state_dim, args.action_dim, args.max_action = 18, 3, 1.6
        self.env = VecSatellites(self.N, device=self.device, d_capture=d_capture,
                                 max_episode_steps=args.max_episode_steps, Flag=self.flag)
        torch.manual_seed(self.seed)                         # same init on every rank
        self.pursuer = PPOLearner(args, "pursuer", self.device, pg=pg, graph_group=args.update_graph_group,
                                  use_graph=use_graphs)
        self.evader = PPOLearner(args, "evader", self.device, pg=pg, graph_group=args.update_graph_group,
                                 use_graph=use_graphs)
        self.learner = self.pursuer if self.flag == 0 else self.evader
        if pg is not None:
            self._broadcast_params()
        self._setup_minibatches(args, pg)
        self.buf = RolloutBuffer(self.T, self.N, self.device)
        self.other_a = torch.zeros((self.N, 3), dtype=torch.float32, device=self.device)
        self.other_lp = torch.zeros((self.N, 3), dtype=torch.float32, device=self.device)
        self.step_base = torch.zeros(1, dtype=torch.int64, device=self.device)   # Philox step offset (u64 bits)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(self.seed * 1000003 + _dist.rank(pg))
        self.use_graphs = use_graphs
        self.chunk = max(1, min(int(args.rollout_graph_chunk), self.T))
        self._graphs = {}
        self._pool = None
        self.iteration_count = 0
        self.rollout_steps = 0
        self.episodes = 0.0
        self.surrogate = None
        self.ellipse_params = None
        if getattr(args, "surrogate", False):
            from .surrogate import Surrogate
            sd = args.surrogate if isinstance(args.surrogate, (str, dict)) else "trained"
            self.surrogate = Surrogate(device=self.device, seed=self.seed, state_dict=sd)
            self.ellipse_params = torch.zeros((self.N, 10), dtype=torch.float32, device=self.device)
        self.env.reset(self.flag, obs_out=self.buf.obs[0])

    STRATA = 8

    def _setup_minibatches(self, args, pg):
        """Local minibatch size and index sampler (see args_param
        dp_minibatch / minibatch_sampler)."""
        W, r = _dist.world_size(pg), _dist.rank(pg)
        mode = getattr(args, "dp_minibatch", "global")
        if mode not in ("global", "per_gpu"):
            raise ValueError("dp_minibatch must be 'global' or 'per_gpu'")
        sampler = getattr(args, "minibatch_sampler", None)
        if sampler is None:
            sampler = "stratified" if (W > 1 and mode == "global") else "uniform"
        if sampler not in ("uniform", "stratified"):
            raise ValueError("minibatch_sampler must be 'uniform' or 'stratified'")
        mb = int(args.mini_batch_size)
        if W > 1 and mode == "global" and sampler != "stratified":
            raise ValueError("global-minibatch data parallelism draws stratified minibatches")
        self.world, self.rank = W, r
        self.dp_minibatch, self.sampler = mode, sampler
        self.global_minibatch = mb if mode == "global" else mb * W
        self.mb_local = mb // W if mode == "global" else mb
        if sampler == "stratified":
            S = self.STRATA
            if S % W or (self.N * W) % S or mb % S or (mode == "global" and mb % W):
                raise ValueError(f"stratified minibatches need world size | {S}, {S} | num_envs*world and "
                                 f"{S} | mini_batch_size (got W={W}, num_envs={self.N}, mb={mb})")
            self.my_strata = list(range(r * (S // W), (r + 1) * (S // W)))
            self.strata_gen = {}
            for s_ in self.my_strata:                # the same stream for a block whatever rank owns it
                g = torch.Generator(device=self.device)
                g.manual_seed(self.seed * 1000003 + 7919 * (s_ + 1))
                self.strata_gen[s_] = g
        for L in (self.pursuer, self.evader):
            L.mini_batch_size = self.mb_local

    def epoch_perm(self):
        """One epoch's minibatch order over the local packed table [T*N]
        (row t*N + j), minibatch-major: the full minibatches of mb_local rows,
        then the tail (BatchSampler drop_last=False)."""
        B = self.T * self.N
        if self.sampler == "uniform":
            return torch.randperm(B, device=self.device, generator=self.gen)
        return stratified_epoch_perm(self.T, self.N, self.world, self.rank, self.global_minibatch, self.strata_gen,
                                     self.STRATA, self.device)

    def _broadcast_params(self):
        # the module parameters are views into each learner's flat P
        _dist.broadcast_([self.pursuer.P, self.evader.P], self.pg)
        self.pursuer.sync_w2t()
        self.evader.sync_w2t()

    # -- rollout ------------------------------------------------------------------
    def _policy_step(self, t, events=None, env=True):
        """One step of CPPO_main.py:121-147 for all envs (no host sync).
        Bench-only knobs: `events` (a pair of torch.cuda.Event) around the env
        step; env=False skips the env step (timing only)."""
        buf = self.buf
        obs_t = buf.obs[t]
        if self.flag == 0:                       # pursuer transitions are stored (CPPO_main.py:141)
            pa, plp, ea, elp = buf.act[t], buf.logp[t], self.other_a, self.other_lp
        else:                                    # evader transitions are stored (CPPO_main.py:210)
            pa, plp, ea, elp = self.other_a, self.other_lp, buf.act[t], buf.logp[t]
        # both agents act on s (CPPO_main.py:122-123): one fused launch, pursuer = agent 0
        policy_act(self.pursuer.H, obs_t, self.pursuer.P, self.evader.P, 1.6, self.seed, self.env_offset, t,
                   pa, plp, ea, elp, step_base=self.step_base)
        if events is not None:
            events[0].record()
        if env:
            self.env.step_autoreset(pa, ea, obs_out=buf.obs[t + 1], reward_out=buf.rew[t], done_out=buf.done[t])
        if events is not None:
            events[1].record()
        if self.surrogate is not None:            # env.ellipse_params of the state the policy sees next
            self.surrogate.env_forward(self.env, out=self.ellipse_params)

    def set_flag(self, flag):
        """Switch the learning agent (Flag 0: pursuer, CPPO_main.py:94-161;
        Flag 1: evader, CPPO_main.py:163-230).  Every env restarts under the
        new Flag; rollout graphs are cached per Flag (they route the learner's
        actions into the buffer)."""
        flag = int(flag)
        if flag not in (0, 1):
            raise ValueError("Flag 0 (pursuer) or 1 (evader)")
        self.flag = flag
        self.learner = self.pursuer if flag == 0 else self.evader
        self.env.reset(flag, obs_out=self.buf.obs[0])

    def self_play(self, phases, iterations_per_phase, timers=None):
        """Alternating training (the reference's Sign == 0 runs
        train_pursuer_network then train_evader_network, CPPO_main.py:336-338):
        `phases` phases of `iterations_per_phase` iterations, starting with the
        current Flag.  Returns the per-iteration statistics."""
        out = []
        for k in range(int(phases)):
            if k:
                self.set_flag(1 - self.flag)
            for _ in range(int(iterations_per_phase)):
                out.append((self.flag, self.iteration(timers)))
        return out

    def _chunk_graph(self, c):
        key = (self.flag, c)
        if key not in self._graphs:
            t0 = c * self.chunk
            t1 = min(self.T, t0 + self.chunk)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            if self._pool is None:
                self._pool = torch.cuda.graph_pool_handle()
            with torch.cuda.graph(g, pool=self._pool):
                for t in range(t0, t1):
                    self._policy_step(t)
            self._graphs[key] = g
        return self._graphs[key]

    def collect(self):
        """T environment steps for all N envs (CPPO_main.py:119-147)."""
        self.step_base.fill_(self.rollout_steps)
        nchunks = (self.T + self.chunk - 1) // self.chunk
        if self.use_graphs:
            if not self._graphs:
                # eager warm-up of one step so lazy allocations happen before capture
                # (restores the env state afterwards)
                f, i = self.env.get_state()
                st = self.env.stats.clone()
                self._policy_step(0)
                self.env.set_state(f, i)
                self.env.stats.copy_(st)
                torch.cuda.synchronize()
            for c in range(nchunks):
                self._chunk_graph(c).replay()
        else:
            for t in range(self.T):
                self._policy_step(t)
        self.rollout_steps += self.T

    # -- learning -----------------------------------------------------------------
    def compute_advantages(self, chunk_steps=64):
        buf, L = self.buf, self.learner
        with torch.no_grad():
            policy_value(L.H, buf.obs.view(-1, 18), L.P, buf.values.view(-1))     # critic(s), all T+1 rows
            gae(buf.rew, buf.done, buf.values, L.gamma, L.lamda, adv_out=buf.adv, vt_out=buf.vtarget)
            adv_n = L.normalize_adv(buf.adv.reshape(-1))
            buf.pack(adv_n)

    def update(self):
        self.learner.update_packed(self.buf.packed, self.episodes, perms=lambda ep: self.epoch_perm())

    def finish_iteration(self):
        # next rollout starts from the current observation
        self.buf.obs[0].copy_(self.buf.obs[self.T])
        st = _dist.sum_(self.env.stats, self.pg)
        self.episodes = float(st[0].item())
        self.iteration_count += 1
        return st.cpu().numpy()

    @property
    def budget_reached(self):
        """True once the finished episodes (all envs, all ranks) reach
        max_train_steps: the reference's loop ends there (CPPO_main.py:110,
        `for epsiode in range(max_train_steps)`), and lr_decay is at 0."""
        return self.episodes >= self.args.max_train_steps

    def train(self, max_iterations=None, timers=None):
        """Iterations until the episode budget (or max_iterations) is reached;
        returns the per-iteration statistics."""
        out = []
        while not self.budget_reached and (max_iterations is None or len(out) < max_iterations):
            out.append(self.iteration(timers))
        return out

    def iteration(self, timers=None):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        self.collect()
        ev[1].record()
        self.compute_advantages()
        ev[2].record()
        self.update()
        ev[3].record()
        if self.learner.comm is not None:
            # RCCL watchdog over the update's graph replays: a dead or stalled
            # peer aborts the communicator and raises instead of hanging here
            self.learner.comm.wait(_dist.dp_timeout_s())
        stats = self.finish_iteration()
        if timers is not None:
            torch.cuda.synchronize()
            timers.setdefault("rollout_ms", []).append(ev[0].elapsed_time(ev[1]))
            timers.setdefault("gae_ms", []).append(ev[1].elapsed_time(ev[2]))
            timers.setdefault("update_ms", []).append(ev[2].elapsed_time(ev[3]))
        return stats
