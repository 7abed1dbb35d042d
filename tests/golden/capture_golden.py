#!/usr/bin/env python3
"""Capture golden input/output vectors from the reference (build container ONLY).

Imports qiaobeibei/PPO-RL-Satellite from /root/reference (read-only) with a
temporary ``gym`` stub (gym is not installed; only ``spaces.Box/Discrete`` are
touched by environment.py:2-4,57,62) and records small .npz fixtures next to
this script.  The reference never travels: the GPU box and every test only
read the committed .npz files.

Run:  python tests/golden/capture_golden.py     (takes ~2-3 minutes)

Fixtures (all seeded, deterministic):
  hybrd_cases.npz     Numerical_iteration_method inputs -> fsolve root
                      (satellite_function.py:558-565), recorded from live
                      env steps plus synthetic draws incl. theta == 0.
  dz_cases.npz        calculate_number_hanger_area inputs -> elements, count
                      (environment.py:317-332, satellite_function.py:18-373)
                      incl. the pursuer states logged in
                      single_pluse_model/spacecraft_state.txt.
  traj_*.npz          environment.step under recorded f32 actions: state
                      before/after every step, obs, reward, done
                      (environment.py:66-255), Flag 0 and Flag 1.
  test_network.npz    CPPO_main.test_network with the one_layer checkpoint,
                      torch/np seed 0 (CPPO_main.py:233-282): per-step obs,
                      actions, log-probs, actor means, rewards, return.
  policy_one_layer.npz one_layer actor/critic weights (data file of the
                      reference, loaded weights_only) + forward outputs.
  update_case.npz     one seeded PPO_continuous.update() (ppo_continuous.py:
                      191-250): buffer, minibatch permutations, adv,
                      v_target, parameters before/after.
  mlpnet2.npz         single_pluse_model/MLPNet2.pth weights + ImprovedNN
                      forward outputs (model.py:7-24), config 5.
"""
import contextlib
import io
import os
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

GYM_STUB = '''
import sys, types
import numpy as _np
class Box:
    def __init__(self, low=None, high=None, shape=None, dtype=_np.float32):
        self.low, self.high, self.dtype = low, high, dtype
        self.shape = tuple(shape) if shape is not None else _np.shape(low)
class Discrete:
    def __init__(self, n):
        self.n = n
spaces = types.ModuleType("gym.spaces")
spaces.Box = Box
spaces.Discrete = Discrete
sys.modules["gym.spaces"] = spaces
'''

MODE = {"int": 0, "int64": 1, "float32": 2, "float64": 3}


def _setup():
    stub = tempfile.mkdtemp(prefix="gymstub_")
    os.makedirs(os.path.join(stub, "gym"))
    with open(os.path.join(stub, "gym", "__init__.py"), "w") as f:
        f.write(GYM_STUB)
    sys.path[:0] = [stub, REF]
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    os.chdir(tempfile.mkdtemp(prefix="refrun_"))


def fuel_mode(v):
    if isinstance(v, (int,)) and not isinstance(v, np.integer):
        return MODE["int"]
    if isinstance(v, np.int64):
        return MODE["int64"]
    if isinstance(v, np.float32):
        return MODE["float32"]
    return MODE["float64"]


def env_state(env):
    return dict(
        Pp=np.asarray(env.Pursuer_position, dtype=np.float64).copy(),
        Pv=np.asarray(env.Pursuer_vector, dtype=np.float64).copy(),
        Ep=np.asarray(env.Escaper_position, dtype=np.float64).copy(),
        Ev=np.asarray(env.Escaper_vector, dtype=np.float64).copy(),
        fuel_c=float(env.fuel_c), fuel_t=float(env.fuel_t), dis=float(env.dis),
        dz=int(env.dangerous_zone), fuel_c_mode=fuel_mode(env.fuel_c), fuel_t_mode=fuel_mode(env.fuel_t),
        vel_int=int(np.asarray(env.Pursuer_vector).dtype.kind == "i" or np.asarray(env.Escaper_vector).dtype.kind == "i"),
        flag=int(env.Flag))


STATE_KEYS = ["Pp", "Pv", "Ep", "Ev", "fuel_c", "fuel_t", "dis", "dz", "fuel_c_mode", "fuel_t_mode", "vel_int", "flag"]


class _GlibcNP(types.ModuleType):
    """numpy proxy whose arccos/arctan/tan are glibc's (math.*) instead of
    numpy's SVML loops; everything else is numpy.  Used to pin the oracle
    bit-exactly: the reference run under this proxy is the reference
    algorithm with glibc libm."""

    def __getattr__(self, k):
        return getattr(np, k)


@contextlib.contextmanager
def glibc_libm(sf):
    import math
    proxy = _GlibcNP("np")
    proxy.arccos = lambda x: np.float64(math.acos(float(x)))
    proxy.arctan = lambda x: np.float64(math.atan(float(x)))
    proxy.tan = lambda x: np.float64(math.tan(float(x)))
    saved = sf.np
    sf.np = proxy
    try:
        yield
    finally:
        sf.np = saved


def _typed_fuel(v, mode):
    return [int(v), np.int64(v), np.float32(v), np.float64(v)][int(mode)]


def set_env_state(env, st):
    vi = bool(st["vel_int"])
    env.Pursuer_position = np.array(st["Pp"], np.int64 if vi else np.float64)   # copies: step() mutates in place
    env.Escaper_position = np.array(st["Ep"], np.int64 if vi else np.float64)
    env.Pursuer_vector = np.array(st["Pv"], np.int64 if vi else np.float64)
    env.Escaper_vector = np.array(st["Ev"], np.int64 if vi else np.float64)
    env.fuel_c = _typed_fuel(st["fuel_c"], st["fuel_c_mode"])
    env.fuel_t = _typed_fuel(st["fuel_t"], st["fuel_t_mode"])
    env.dis = float(st["dis"])
    env.dangerous_zone = int(st["dz"])
    env.Flag = int(st["flag"])


class Recorder:
    """Wraps Numerical_iteration_method / calculate_number_hanger_area."""

    def __init__(self, sf, environment):
        self.hyb = []
        self.dz = []
        orig_nim = sf.Time_window_of_danger_zone.Numerical_iteration_method
        orig_dz = environment.satellites.calculate_number_hanger_area
        rec = self

        def nim(obj, Delta_Vm, theta, v_1x, v_1y, h, alpha_guess):
            res = orig_nim(obj, Delta_Vm, theta, v_1x, v_1y, h, alpha_guess)
            rec.hyb.append([float(Delta_Vm), float(theta), float(v_1x), float(v_1y), float(h),
                            float(alpha_guess), float(res)])
            return res

        def dzf(envself):
            Rc, Vc = envself.relative_state_to_absolute_state(envself.Pursuer_position, envself.Pursuer_vector)
            Rt, Vt = envself.relative_state_to_absolute_state(envself.Escaper_position, envself.Escaper_vector)
            fc = envself.fuel_c
            out = orig_dz(envself)
            rec.dz.append((np.concatenate([Rc, Vc, Rt, Vt]).astype(np.float64), float(fc), fuel_mode(fc),
                           int(envself.dangerous_zone)))
            return out

        sf.Time_window_of_danger_zone.Numerical_iteration_method = nim
        environment.satellites.calculate_number_hanger_area = dzf


def run_traj(environment, args, seed, n_steps, flag, d_capture, policy, max_ep):
    import torch
    torch.manual_seed(seed)
    np.random.seed(seed)
    args.max_episode_steps = max_ep
    env = environment.satellites(args=args)
    env.d_capture = d_capture
    rng = np.random.default_rng(seed)
    recs = {k: [] for k in ["pa", "ea", "count", "obs", "r", "done"] + ["b_" + k for k in STATE_KEYS] +
            ["a_" + k for k in STATE_KEYS]}
    s = env.reset(flag)
    count = 0
    for t in range(n_steps):
        count += 1
        pa, ea = policy(rng, s, t)
        st = env_state(env)
        with contextlib.redirect_stdout(io.StringIO()):
            s_, r, done = env.step(pa, ea, count)
        st2 = env_state(env)
        recs["pa"].append(np.asarray(pa, np.float32)); recs["ea"].append(np.asarray(ea, np.float32))
        recs["count"].append(count); recs["obs"].append(np.asarray(s_, np.float64)); recs["r"].append(float(r))
        recs["done"].append(int(done))
        for k in STATE_KEYS:
            recs["b_" + k].append(st[k]); recs["a_" + k].append(st2[k])
        s = s_
        if done:
            s = env.reset(flag)
            count = 0
    out = {k: np.asarray(v) for k, v in recs.items()}
    # same before-states and actions, reference run with glibc arccos/arctan/tan
    import satellite_function as sf
    dz_g, r_g = [], []
    with glibc_libm(sf):
        for t in range(len(out["r"])):
            set_env_state(env, {k: out["b_" + k][t] for k in STATE_KEYS})
            with contextlib.redirect_stdout(io.StringIO()):
                _, r, _ = env.step(out["pa"][t], out["ea"][t], int(out["count"][t]))
            dz_g.append(int(env.dangerous_zone)); r_g.append(float(r))
    out["a_dz_glibc"] = np.asarray(dz_g)
    out["r_glibc"] = np.asarray(r_g)
    out["meta"] = np.array([seed, flag, d_capture, max_ep, n_steps], dtype=np.float64)
    return out


def main():
    _setup()
    import torch
    torch.set_num_threads(1)
    import satellite_function as sf
    import environment
    import CPPO_main
    import ppo_continuous
    import replaybuffer
    from torch.utils.data.sampler import BatchSampler, SubsetRandomSampler

    rec = Recorder(sf, environment)
    args = CPPO_main.args_param(chkpt_dir=os.path.join(REF, "model_file", "one_layer"))

    # ---------------- trajectories -----------------------------------------
    def uniform(rng, s, t):
        return (rng.uniform(-1.6, 1.6, 3).astype(np.float32), rng.uniform(-1.6, 1.6, 3).astype(np.float32))

    def wide(rng, s, t):   # exercises clipping and exact zero components
        pa = rng.uniform(-2.5, 2.5, 3).astype(np.float32)
        ea = rng.uniform(-2.5, 2.5, 3).astype(np.float32)
        if t % 7 == 3:
            pa[rng.integers(3)] = 0.0
        if t % 11 == 5:
            ea[:] = 0.0
        return pa, ea

    def chase(rng, s, t):  # PD pursuit: reaches d_range, freezes, captures
        rel = np.asarray(s[0:3], np.float64)
        vrel = np.asarray(s[3:6], np.float64)
        a = -2e-4 * rel - 0.08 * vrel + rng.normal(0, 0.05, 3)
        pa = np.clip(a, -1.6, 1.6).astype(np.float32)
        ea = rng.uniform(-0.3, 0.3, 3).astype(np.float32)
        return pa, ea

    trajs = [
        ("traj_uniform_f0", dict(seed=1, n_steps=1200, flag=0, d_capture=15000.0, policy=uniform, max_ep=400)),
        ("traj_wide_f0", dict(seed=2, n_steps=800, flag=0, d_capture=20000.0, policy=wide, max_ep=300)),
        ("traj_chase_f0", dict(seed=3, n_steps=1500, flag=0, d_capture=15000.0, policy=chase, max_ep=1000)),
        ("traj_uniform_f1", dict(seed=4, n_steps=800, flag=1, d_capture=15000.0, policy=uniform, max_ep=300)),
        ("traj_chase_f1", dict(seed=5, n_steps=1200, flag=1, d_capture=20000.0, policy=chase, max_ep=1000)),
    ]
    for name, kw in trajs:
        d = run_traj(environment, args, **kw)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **d)
        print(name, "steps", len(d["r"]), "dones", int(d["done"].sum()), "dz>0", int((d["a_dz"] > 0).sum()),
              "frozen-ish", int(((d["b_dis"] < 1e5) & (d["b_dz"] != 0)).sum()),
              "fuel modes", np.unique(d["a_fuel_c_mode"]).tolist())

    # ---------------- test_network (seed 0, one_layer ckpt) -----------------
    tn = {}
    for max_ep in (64, 1000):
        torch.manual_seed(0)
        np.random.seed(0)
        a2 = CPPO_main.args_param(max_episode_steps=max_ep, batch_size=64, max_train_steps=5000, K_epochs=3,
                                  chkpt_dir=os.path.join(REF, "model_file", "one_layer"))
        env = environment.satellites(Pursuer_position=np.array([2000000, 2000000, 1000000]),
                                     Pursuer_vector=np.array([1710, 1140, 1300]),
                                     Escaper_position=np.array([1850000, 2000000, 1000000]),
                                     Escaper_vector=np.array([1710, 1140, 1300]), d_capture=50000, args=a2)
        log = {"obs_in": [], "pa": [], "ea": [], "plogp": [], "pmean": [], "r": [], "done": []}
        orig_choose = ppo_continuous.PPO_continuous.choose_action

        def choose(self, s, _orig=orig_choose, _log=log):
            a, lp = _orig(self, s)
            if self is _log.get("_pursuer"):
                with torch.no_grad():
                    m = self.actor(torch.unsqueeze(torch.tensor(s, dtype=torch.float), 0)).numpy().ravel()
                _log["obs_in"].append(np.asarray(s, np.float64)); _log["pa"].append(a); _log["plogp"].append(lp)
                _log["pmean"].append(m)
            else:
                _log["ea"].append(a)
            return a, lp

        orig_init = ppo_continuous.PPO_continuous.__init__

        def init(self, args_, idx, _orig=orig_init, _log=log):
            _orig(self, args_, idx)
            if idx == "pursuer":
                _log["_pursuer"] = self

        orig_step = environment.satellites.step

        def step(self, pa, ea, c, _orig=orig_step, _log=log):
            s_, r, d = _orig(self, pa, ea, c)
            _log["r"].append(float(r)); _log["done"].append(int(d))
            return s_, r, d

        ppo_continuous.PPO_continuous.choose_action = choose
        ppo_continuous.PPO_continuous.__init__ = init
        environment.satellites.step = step
        with contextlib.redirect_stdout(io.StringIO()) as buf:
            CPPO_main.test_network(a2, env, show_pictures=False, d_capture=20000)
        ppo_continuous.PPO_continuous.choose_action = orig_choose
        ppo_continuous.PPO_continuous.__init__ = orig_init
        environment.satellites.step = orig_step
        ret = 0.0
        for _r in log["r"]:
            ret += _r   # same float order as CPPO_main.py:264
        print("test_network max_ep", max_ep, "return", repr(ret), "| printed:", buf.getvalue().strip().splitlines()[-1])
        for k in ("obs_in", "pa", "ea", "plogp", "pmean", "r", "done"):
            tn[f"{k}_{max_ep}"] = np.asarray(log[k])
        tn[f"return_{max_ep}"] = np.array(ret)
    np.savez_compressed(os.path.join(OUT, "test_network.npz"), **tn)

    # ---------------- policy weights + forward --------------------------------
    sd_a = torch.load(os.path.join(REF, "model_file/one_layer/agent_pursuer_actor_Gaussian"), weights_only=True,
                      map_location="cpu")
    sd_c = torch.load(os.path.join(REF, "model_file/one_layer/agent_pursuer_critic"), weights_only=True,
                      map_location="cpu")
    a3 = CPPO_main.args_param(chkpt_dir="/nonexistent")
    a3.state_dim, a3.action_dim, a3.max_action = 18, 3, 1.6
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        actor = ppo_continuous.Actor_Gaussian(a3, "pursuer")
        critic = ppo_continuous.Critic(a3, "pursuer")
    actor.load_state_dict(sd_a)
    critic.load_state_dict(sd_c)
    rng = np.random.default_rng(7)
    obs = np.concatenate([tn["obs_in_1000"][:200].astype(np.float32),
                          (rng.standard_normal((56, 18)) * rng.uniform(0.1, 3e5, (56, 18))).astype(np.float32),
                          rng.uniform(-2, 2, (64, 18)).astype(np.float32)])
    with torch.no_grad():
        o = torch.tensor(obs)
        mean = actor(o).numpy()
        v = critic(o).numpy()
        dist = actor.get_dist(o)
        act = torch.clamp(dist.sample(), -1.6, 1.6)
        logp = dist.log_prob(act).numpy()
        ent = dist.entropy().numpy()
    pol = {"obs": obs, "mean": mean, "value": v, "act": act.numpy(), "logp": logp, "entropy": ent}
    for k, t in sd_a.items():
        pol["actor." + k] = t.numpy()
    for k, t in sd_c.items():
        pol["critic." + k] = t.numpy()
    np.savez_compressed(os.path.join(OUT, "policy_one_layer.npz"), **pol)

    # ---------------- one seeded update() --------------------------------------
    torch.manual_seed(123)
    np.random.seed(123)
    a4 = CPPO_main.args_param(batch_size=512, mini_batch_size=64, hidden_width=64, K_epochs=3,
                              max_train_steps=1000, chkpt_dir="/nonexistent")
    a4.state_dim, a4.action_dim, a4.max_action = 18, 3, 1.6
    with contextlib.redirect_stdout(io.StringIO()):
        agent = ppo_continuous.PPO_continuous(a4, "pursuer")
    p0 = {("actor." + k): v.detach().clone().numpy() for k, v in agent.actor.state_dict().items()}
    p0.update({("critic." + k): v.detach().clone().numpy() for k, v in agent.critic.state_dict().items()})
    buf = replaybuffer.ReplayBuffer(a4)
    a4.max_episode_steps = 100
    env = environment.satellites(args=a4)
    env.d_capture = 15000
    s = env.reset(0)
    cnt = 0
    for t in range(a4.batch_size):
        cnt += 1
        pa, plp = agent.choose_action(s)
        ea = np.random.uniform(-1.6, 1.6, 3).astype(np.float32)
        with contextlib.redirect_stdout(io.StringIO()):
            s_, r, done = env.step(pa, ea, cnt)
        dw = bool(done or cnt >= a4.max_episode_steps)
        buf.store(s, pa, plp, r, s_, dw, done)
        s = s_
        if done:
            s = env.reset(0)
            cnt = 0
    S, A, LP, R, S_, DW, DONE = buf.numpy_to_tensor()
    with torch.no_grad():
        vs = agent.critic(S).numpy()
        vs_ = agent.critic(S_).numpy()
    rng_state = torch.get_rng_state()
    perms = []
    for _ in range(a4.K_epochs):
        perms.append(np.concatenate([np.asarray(ix) for ix in BatchSampler(SubsetRandomSampler(range(a4.batch_size)),
                                                                              a4.mini_batch_size, False)]))
    torch.set_rng_state(rng_state)
    # replicate adv / v_target exactly as update() does (ppo_continuous.py:198-210)
    adv = []
    gae = 0
    with torch.no_grad():
        deltas = R + agent.gamma * (1.0 - DW) * torch.tensor(vs_) - torch.tensor(vs)
        for delta, d in zip(reversed(deltas.flatten().numpy()), reversed(DONE.flatten().numpy())):
            gae = delta + agent.gamma * agent.lamda * gae * (1.0 - d)
            adv.insert(0, gae)
        adv = torch.tensor(adv, dtype=torch.float).view(-1, 1)
        v_target = adv + torch.tensor(vs)
        adv_n = ((adv - adv.mean()) / (adv.std() + 1e-5))
    total_steps = 37
    agent.update(buf, total_steps)
    p1 = {("actor." + k): v.detach().clone().numpy() for k, v in agent.actor.state_dict().items()}
    p1.update({("critic." + k): v.detach().clone().numpy() for k, v in agent.critic.state_dict().items()})
    upd = {"s": S.numpy(), "a": A.numpy(), "logp": LP.numpy(), "r": R.numpy(), "s_": S_.numpy(), "dw": DW.numpy(),
           "done": DONE.numpy(), "vs": vs, "vs_": vs_, "adv": adv.numpy(), "v_target": v_target.numpy(),
           "adv_norm": adv_n.numpy(), "perms": np.stack(perms), "total_steps": np.array(total_steps),
           "hp": np.array([a4.batch_size, a4.mini_batch_size, a4.hidden_width, a4.K_epochs, a4.max_train_steps,
                           a4.lr_a, a4.lr_c, a4.gamma, a4.lamda, a4.epsilon, a4.entropy_coef]),
           "lr_after": np.array([agent.optimizer_actor.param_groups[0]["lr"],
                                 agent.optimizer_critic.param_groups[0]["lr"]])}
    for k, v in p0.items():
        upd["p0." + k] = v
    for k, v in p1.items():
        upd["p1." + k] = v
    np.savez_compressed(os.path.join(OUT, "update_case.npz"), **upd)
    print("update_case: B", a4.batch_size, "adv mean", float(adv.mean()), "dones", int(DONE.sum()))

    # ---------------- hybrd / dz cases ------------------------------------------
    hyb = np.asarray(rec.hyb, dtype=np.float64)
    # synthetic draws around the live distribution, incl. theta == 0 and random guesses
    rng = np.random.default_rng(11)
    live = hyb[rng.choice(len(hyb), size=min(len(hyb), 6000), replace=False)]
    syn = []

    class Dummy:
        u = 3.986e14
    nim = sf.Time_window_of_danger_zone.Numerical_iteration_method
    for k in range(8000):
        base = hyb[rng.integers(len(hyb))]
        dvm = base[0] * rng.uniform(0.2, 3.0)
        theta = 0.0 if k % 50 == 0 else rng.uniform(0, 2 * np.pi)
        v1x = base[2] * rng.uniform(0.5, 1.5) + rng.normal(0, 50)
        v1y = base[3] * rng.uniform(0.9, 1.1)
        h = base[4] * rng.uniform(0.9, 1.1)
        guess = [np.pi / 2, -np.pi / 2][k % 2] if k % 5 else rng.uniform(-4, 4)
        syn.append([dvm, theta, v1x, v1y, h, guess])
    rec.hyb = []
    for row in syn:
        nim(Dummy(), *row)
    syn_out = np.asarray(rec.hyb)
    np.savez_compressed(os.path.join(OUT, "hybrd_cases.npz"), live=live, synthetic=syn_out)
    print("hybrd cases: live", len(live), "synthetic", len(syn_out))

    dz = rec.dz
    X = np.stack([d[0] for d in dz])
    fuel = np.array([d[1] for d in dz])
    mode = np.array([d[2] for d in dz], dtype=np.int32)
    cnt = np.array([d[3] for d in dz], dtype=np.int32)
    sel = rng.choice(len(X), size=min(len(X), 4000), replace=False)
    X, fuel, mode, cnt = X[sel], fuel[sel], mode[sel], cnt[sel]
    # spacecraft_state.txt pursuer states (environment.py:321 log) against logged-run targets
    txt = open(os.path.join(REF, "single_pluse_model/spacecraft_state.txt"), encoding="utf-8-sig").read()
    parts = [p for p in txt.split("R0_c, V0_c, fuel_c:") if p.strip()]
    Xs, fs = [], []
    for p in parts:
        p = p.replace("[", " ").replace("]", " ")
        vals = [float(v) for v in p.split()]
        if len(vals) == 7:
            Xs.append(vals[:6]); fs.append(vals[6])
    Xs = np.asarray(Xs)
    tgt = X[rng.integers(len(X), size=len(Xs)), 6:12]
    elems_c, elems_t, cnt2 = [], [], []
    for i in range(len(Xs)):
        twd = sf.Time_window_of_danger_zone(R0_c=Xs[i, :3].copy(), V0_c=Xs[i, 3:6].copy(), R0_t=tgt[i, :3].copy(),
                                            V0_t=tgt[i, 3:].copy(), Delta_V_c=float(fs[i]), time_step=1)
        cnt2.append(twd.calculate_number_of_hanger_area())
    Xtxt = np.concatenate([Xs, tgt], axis=1)
    allX = np.concatenate([X, Xtxt])
    allfuel = np.concatenate([fuel, np.asarray(fs)])
    allmode = np.concatenate([mode, np.full(len(Xs), 3, np.int32)])
    allcnt = np.concatenate([cnt, np.asarray(cnt2, np.int32)])
    for i in range(len(allX)):
        ec = sf.Time_window_of_danger_zone.calculate_orbital_elements(3.986e14, allX[i, 0:3], allX[i, 3:6])
        et = sf.Time_window_of_danger_zone.calculate_orbital_elements(3.986e14, allX[i, 6:9], allX[i, 9:12])
        elems_c.append(ec); elems_t.append(et)
    cnt_g, ec_g, et_g = [], [], []
    with glibc_libm(sf):
        for i in range(len(allX)):
            twd = sf.Time_window_of_danger_zone(R0_c=allX[i, 0:3].copy(), V0_c=allX[i, 3:6].copy(),
                                                R0_t=allX[i, 6:9].copy(), V0_t=allX[i, 9:12].copy(),
                                                Delta_V_c=_typed_fuel(allfuel[i], allmode[i]), time_step=1)
            cnt_g.append(twd.calculate_number_of_hanger_area())
            ec_g.append([twd.a_c, twd.e_c, twd.i_c, twd.omega_c, twd.Omega_c, twd.f0_c])
            et_g.append([twd.a_t, twd.e_t, twd.i_t, twd.omega_t, twd.Omega_t, twd.f0_t])
    np.savez_compressed(os.path.join(OUT, "dz_cases.npz"), X=allX, fuel=allfuel, mode=allmode, count=allcnt,
                        elems_c=np.asarray(elems_c, np.float64), elems_t=np.asarray(elems_t, np.float64),
                        count_glibc=np.asarray(cnt_g, np.int32), elems_c_glibc=np.asarray(ec_g, np.float64),
                        elems_t_glibc=np.asarray(et_g, np.float64), n_txt=np.array(len(Xs)))
    print("dz glibc-vs-svml count flips:", int((np.asarray(cnt_g) != allcnt).sum()))
    print("dz cases", len(allX), "count hist", np.bincount(allcnt).tolist())

    # ---------------- config 5: ImprovedNN + MLPNet2.pth -------------------------
    from single_pluse_model import model as spm
    sd = torch.load(os.path.join(REF, "single_pluse_model/MLPNet2.pth"), weights_only=True, map_location="cpu")
    net = spm.ImprovedNN()
    net.load_state_dict(sd)
    net.eval()
    feats = []
    for i in range(len(allX)):
        el = sf.Time_window_of_danger_zone.calculate_orbital_elements(3.986e14, allX[i, 0:3], allX[i, 3:6])
        feats.append([el[0], el[1], el[2], el[5], allfuel[i]])    # real_time_data_process.py:114-116
    feats = np.asarray(feats, np.float32)[:512]
    with torch.no_grad():
        y = net(torch.tensor(feats)).numpy()
        y0 = net(torch.zeros(4, 5)).numpy()
    mm = {"x": feats, "y": y, "y_zero": y0}
    for k, t in sd.items():
        mm[k] = t.numpy()
    np.savez_compressed(os.path.join(OUT, "mlpnet2.npz"), **mm)
    print("mlpnet2: |y|max", float(np.abs(y).max()), "|y(0)|max", float(np.abs(y0).max()))


if __name__ == "__main__":
    main()
