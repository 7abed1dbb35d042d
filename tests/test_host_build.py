"""The host build of the product's env ABI (include/satenv_cpu.h) and the
drop-in on device="cpu" -- BASELINE.json configs[0] (CPPO_main on CPU, no
GPU) -- against the reference.  CPU only.

The host build is the env kernels' own FP64 source (csrc/satenv_device.h,
satenv_step.h) compiled by g++, with glibc transcendentals; the reference
run with glibc libm is what the *_glibc fixture keys hold, so the bar here
is bit-exact everywhere: obs, state planes, done, danger-zone counts and
rewards.  The agents on device="cpu" are the same nn.Modules stepped by
torch's CPU autograd / Adam (satrl.ppo.HostLearner), so the closed loop --
env + agents + RNG order -- reproduces the reference's unforced episodes and
training loop exactly (closed_loop.npz, train_loop.npz).
"""
import contextlib
import io
import os

import numpy as np
import pytest
import torch

from conftest import TRAJ_NAMES, golden


def _planes(d, prefix, idx):
    from satrl.env import pack_bits
    f = np.stack([d[prefix + "Pp"][idx, 0], d[prefix + "Pp"][idx, 1], d[prefix + "Pp"][idx, 2],
                  d[prefix + "Pv"][idx, 0], d[prefix + "Pv"][idx, 1], d[prefix + "Pv"][idx, 2],
                  d[prefix + "Ep"][idx, 0], d[prefix + "Ep"][idx, 1], d[prefix + "Ep"][idx, 2],
                  d[prefix + "Ev"][idx, 0], d[prefix + "Ev"][idx, 1], d[prefix + "Ev"][idx, 2],
                  d[prefix + "fuel_c"][idx], d[prefix + "fuel_t"][idx], d[prefix + "dis"][idx]]).astype(np.float64)
    bits = np.array([pack_bits(a, b, c, e) for a, b, c, e in zip(d[prefix + "fuel_c_mode"][idx],
                                                                  d[prefix + "fuel_t_mode"][idx],
                                                                  d[prefix + "vel_int"][idx], d[prefix + "flag"][idx])])
    i = np.stack([d[prefix + "dz"][idx], d["count"][idx], bits]).astype(np.int32)
    return torch.from_numpy(np.ascontiguousarray(f)), torch.from_numpy(np.ascontiguousarray(i))


@pytest.mark.parametrize("name", TRAJ_NAMES)
def test_host_step_bitexact_vs_reference(name):
    """Every recorded step as one env of a single satenv_cpu_step call:
    obs, state planes, done, count and reward equal the glibc reference."""
    from satrl.env import VecSatellites
    d = golden(name)
    _, flag, dcap, maxep, _ = d["meta"]
    n = len(d["r"])
    env = VecSatellites(n, device="cpu", d_capture=float(dcap), max_episode_steps=int(maxep), Flag=int(flag))
    env.set_state(*_planes(d, "b_", np.arange(n)))
    obs64 = torch.empty((n, 18), dtype=torch.float64)
    _, r, done = env.step(torch.tensor(d["pa"], dtype=torch.float32), torch.tensor(d["ea"], dtype=torch.float32),
                          torch.tensor(d["count"], dtype=torch.int32), obs64_out=obs64)
    assert env.check_errors() == 0
    fa, ia = env.get_state()
    fr, ir = _planes(d, "a_", np.arange(n))
    assert np.array_equal(obs64.numpy(), d["obs"])
    assert np.array_equal(done.numpy(), d["done"])
    assert torch.equal(fa, fr) and torch.equal(ia[2], ir[2])
    assert np.array_equal(ia[0].numpy(), d["a_dz_glibc"])
    assert np.array_equal(r.numpy(), d["r_glibc"])


def _cw_ode_pairs(g, a):
    """env k = (pursuer x0[2k], evader x0[2k+1]) of cw_ode.npz case a"""
    x0, out = g["x0"], g["out"][a]
    n = (len(x0) + 1) // 2
    ip = np.arange(n) * 2
    ie = np.minimum(ip + 1, len(x0) - 1)
    f = np.zeros((15, n))
    f[0:6] = x0[ip].T
    f[6:12] = x0[ie].T
    f[12:14] = 320.0
    f[14] = np.inf
    i32 = np.zeros((3, n), np.int32)
    from satrl.env import pack_bits
    i32[2] = pack_bits(0, 0, 0, 0)
    want = np.concatenate([out[ip].T, out[ie].T])
    return n, torch.from_numpy(f), torch.from_numpy(i32), want


def test_host_propagator2_is_the_reference_solve_ivp():
    """propagator 2 (satellite_function.py:783-839, solve_ivp RK45 over the
    100-s step) in the host build: zero actions, every captured state pair
    propagated bit for bit like the reference's numerical_calculation(100)."""
    from satrl.env import VecSatellites
    g = golden("cw_ode")
    a = list(g["t"]).index(100.0)
    n, f, i32, want = _cw_ode_pairs(g, a)
    env = VecSatellites(n, device="cpu", d_capture=0.0, max_episode_steps=1000, propagator=2)
    env.set_state(f, i32)
    z = torch.zeros((n, 3), dtype=torch.float32)
    env.step(z, z, torch.ones(n, dtype=torch.int32))
    assert env.check_errors() == 0
    fa, _ = env.get_state()
    assert np.array_equal(fa[0:12].numpy(), want)


def test_host_danger_zone_counts_exact():
    import ctypes as C
    from satrl import _lib
    d = golden("dz_cases")
    n = len(d["X"])
    X = np.ascontiguousarray(d["X"], np.float64)
    fuel = np.ascontiguousarray(d["fuel"], np.float64)
    mode = np.ascontiguousarray(d["mode"], np.int32)
    out = np.zeros(n, np.int32)
    vp = C.c_void_p
    _lib.check(_lib.lib().satenv_cpu_danger_zone(n, X.ctypes.data_as(vp), fuel.ctypes.data_as(vp),
                                                 mode.ctypes.data_as(vp), out.ctypes.data_as(vp), None),
               "satenv_cpu_danger_zone")
    assert np.array_equal(out, d["count_glibc"])


def test_host_autoreset_matches_oracle(oracle):
    """satenv_cpu_step_autoreset (8 threads) over 256 envs x 200 steps from
    reset == the oracle's batched replay: done and f32 rewards identical."""
    from satrl.env import VecSatellites
    n, T = 256, 200
    rng = np.random.default_rng(11)
    pa = rng.uniform(-1.6, 1.6, (T, n, 3)).astype(np.float32)
    ea = rng.uniform(-1.6, 1.6, (T, n, 3)).astype(np.float32)
    rew_o, done_o = oracle.rollout(n, T, pa, ea, d_capture=15000.0, max_episode_steps=80, nthreads=4)
    env = VecSatellites(n, device="cpu", d_capture=15000.0, max_episode_steps=80, threads=8)
    env.reset(0)
    for t in range(T):
        _, r, dn = env.step_autoreset(torch.from_numpy(pa[t]), torch.from_numpy(ea[t]))
        assert np.array_equal(dn.numpy(), done_o[t]), t
        assert np.array_equal(r.numpy(), rew_o[t].astype(np.float32)), t
    assert env.stats[0].item() == done_o.sum()


def test_host_requires_host_tensors_and_is_only_used_when_asked():
    from satrl import _lib
    from satrl.env import VecSatellites
    env = VecSatellites(4, device="cpu")
    with pytest.raises(_lib.NativeError):
        env.step(torch.zeros((4, 3), dtype=torch.float64), torch.zeros((4, 3)))
    if not torch.cuda.is_available():
        with pytest.raises(_lib.NativeError):
            VecSatellites(4)                     # the default device never falls back to the host build


def _one_layer_ckpt(d):
    g = golden("policy_one_layer")
    for net, fname in (("actor", "agent_pursuer_actor_Gaussian"), ("critic", "agent_pursuer_critic")):
        torch.save({k[len(net) + 1:]: torch.tensor(g[k]) for k in g.files if k.startswith(net + ".")},
                   os.path.join(d, fname))


def _main_env(args):
    from satrl.env import satellites
    return satellites(Pursuer_position=np.array([2000000, 2000000, 1000000]),
                      Pursuer_vector=np.array([1710, 1140, 1300]),
                      Escaper_position=np.array([1850000, 2000000, 1000000]),
                      Escaper_vector=np.array([1710, 1140, 1300]), d_capture=50000, args=args, device="cpu")


@pytest.mark.parametrize("max_ep", [64, 1000])
def test_host_closed_loop_test_network_is_the_reference(tmp_path, max_ep):
    """CPPO_main.test_network, UNFORCED, on device="cpu" (host env build +
    torch-CPU agents), seeded as SURVEY.md §3.2: every reward, done and the
    printed return equal the reference's clean run (closed_loop.npz:
    12.694102317688985 at 64 steps, -1490.0011561101467 at 1000)."""
    from satrl import env as E
    from satrl.trainer import args_param, test_network
    g = golden("closed_loop")
    _one_layer_ckpt(str(tmp_path))
    rs, ds = [], []
    orig = E.satellites.step

    def step(self, pa, ea, c):
        s_, r, d = orig(self, pa, ea, c)
        rs.append(r)
        ds.append(int(d))
        return s_, r, d

    E.satellites.step = step
    try:
        torch.manual_seed(0)
        np.random.seed(0)
        a2 = args_param(max_episode_steps=max_ep, batch_size=64, max_train_steps=5000, K_epochs=3,
                        chkpt_dir=str(tmp_path), device="cpu")
        with contextlib.redirect_stdout(io.StringIO()):
            ret = test_network(a2, _main_env(a2), show_pictures=False, d_capture=20000)
    finally:
        E.satellites.step = orig
    assert np.array_equal(np.asarray(rs, np.float64), g[f"r_{max_ep}"])
    assert np.array_equal(np.asarray(ds, np.uint8), g[f"done_{max_ep}"])
    assert ret == float(g[f"return_{max_ep}"])
    assert ret == {64: 12.694102317688985, 1000: -1490.0011561101467}[max_ep]


def test_host_training_loop_is_the_reference(tmp_path):
    """CPPO_main.train_pursuer_network as the reference's __main__ runs it
    (Sign 0: pre-trained one_layer pursuer, batch 64, K_epochs 3, d_capture
    15000), seed 0, 3 episodes, UNFORCED on device="cpu": every reward and
    done, every sampled action, and the pursuer's parameters after each of
    the 3 updates equal the reference's (train_loop.npz, capture_train.py,
    one torch thread as captured)."""
    from satrl import env as E
    from satrl import ppo as P
    from satrl.trainer import args_param, train_pursuer_network
    g = golden("train_loop")
    _one_layer_ckpt(str(tmp_path))
    log = {"r": [], "done": [], "pa": []}
    after = []
    orig_step, orig_update, orig_choose = E.satellites.step, P.PPO_continuous.update, P.PPO_continuous.choose_action
    agents = {}

    def step(self, pa, ea, c):
        s_, r, d = orig_step(self, pa, ea, c)
        log["r"].append(float(r))
        log["done"].append(int(d))
        log["pa"].append(np.asarray(pa))
        return s_, r, d

    def update(self, rb, total_steps):
        orig_update(self, rb, total_steps)
        after.append({f"{net}.{k}": v.detach().numpy().copy() for net in ("actor", "critic")
                      for k, v in getattr(self, net).state_dict().items()})

    nthreads = torch.get_num_threads()
    E.satellites.step, P.PPO_continuous.update = step, update
    try:
        torch.set_num_threads(1)
        torch.manual_seed(0)
        np.random.seed(0)
        args = args_param(max_episode_steps=64, batch_size=64, max_train_steps=3, K_epochs=3, chkpt_dir=str(tmp_path),
                          device="cpu")
        env = _main_env(args)
        train_pursuer_network(args, env, show_picture=False, pre_train=True, d_capture=15000, max_episodes=3)
    finally:
        E.satellites.step, P.PPO_continuous.update, P.PPO_continuous.choose_action = (orig_step, orig_update,
                                                                                    orig_choose)
        torch.set_num_threads(nthreads)
    n = len(g["r"])
    assert len(log["r"]) == n
    assert np.array_equal(np.asarray(log["r"]), g["r"])
    assert np.array_equal(np.asarray(log["done"]), g["done"])
    assert np.array_equal(np.asarray(log["pa"], np.float32), g["pa"].astype(np.float32))
    assert len(after) == int(g["n_updates"])
    for k, got in enumerate(after):
        for name, v in got.items():
            assert np.array_equal(v, g[f"after{k}.{name}"]), (k, name, float(np.abs(v - g[f"after{k}.{name}"]).max()))
