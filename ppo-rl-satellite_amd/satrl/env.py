"""Environment front-ends over the HIP C-ABI (include/satenv.h).

* ``VecSatellites`` -- N environments resident in HBM, torch device tensors in
  and out; the engine's rollout path.
* ``satellites``    -- drop-in for the reference class
  (qiaobeibei/PPO-RL-Satellite environment.py:8-413): same constructor
  keywords, ``reset(Flag)`` / ``step(pursuer_action, escaper_action,
  epsiode_count)`` signatures, numpy outputs with the reference's dtypes and
  the attributes its callers read (``observation_space``, ``action_space``,
  ``d_capture`` ...).  It runs one env on the GPU kernel.

Both run on the host build of the same env ABI (include/satenv_cpu.h: the
step source compiled by g++, OpenMP over envs) when asked with
device="cpu" -- BASELINE.json configs[0], CPPO_main on a machine without a
GPU.  Nothing falls back to it: without a GPU the default device raises.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np
import torch

from . import _lib
from ._lib import ACT_DIM, OBS_DIM, SATENV_F64_PLANES, SATENV_I32_PLANES, check, ptr, require_cpu, require_cuda, stream_ptr

PYINT, I64, F32, F64 = 0, 1, 2, 3
STATE_F64 = ["Pp0", "Pp1", "Pp2", "Pv0", "Pv1", "Pv2", "Ep0", "Ep1", "Ep2", "Ev0", "Ev1", "Ev2",
             "fuel_c", "fuel_t", "dis"]
STATE_I32 = ["dz", "episode_count", "bits"]


def default_params(**overrides) -> _lib.SatenvParams:
    p = _lib.SatenvParams()
    check(_lib.lib().satenv_default_params(C.byref(p)), "satenv_default_params")
    names = {f[0] for f in _lib.SatenvParams._fields_}
    for k, v in overrides.items():
        if k not in names:
            raise TypeError(f"unknown satenv parameter {k!r} (include/satenv.h satenv_params)")
        if k in ("R_cw", "V_cw", "stm", "init_kin"):
            getattr(p, k)[:] = [float(x) for x in np.asarray(v, dtype=np.float64).ravel()]
        else:
            setattr(p, k, v)
    return p


def stm(t: float = 100.0) -> np.ndarray:
    out = (C.c_double * 36)()
    check(_lib.lib().satenv_stm(float(t), out), "satenv_stm")
    return np.array(out[:]).reshape(6, 6)


def rk4_j2(rv, h, steps, out=None):
    """RK4 two-body + J2 propagation of 轨道外推-龙格库塔算法.py (km, km/s) for a
    batch of states rv [n][6] (f64, CUDA): `steps` steps of h seconds on the
    satenv_rk4_j2 kernel (one lane per state, SoA planes internally)."""
    n = rv.shape[0]
    _lib.require_cuda(rv, torch.float64, (n, 6), "rv")
    soa = rv.t().contiguous()
    check(_lib.lib().satenv_rk4_j2(n, ptr(soa), float(h), int(steps), ptr(soa), stream_ptr()), "satenv_rk4_j2")
    res = soa.t()
    if out is None:
        return res.contiguous()
    out.copy_(res)
    return out


def _num_mode(v) -> int:
    if isinstance(v, np.float32):
        return F32
    if isinstance(v, (np.floating, float)):
        return F64
    if isinstance(v, np.integer):
        return I64
    return PYINT


class Box:
    """Minimal stand-in for ``gym.spaces.Box`` (environment.py:57): shape/low/high/dtype."""

    def __init__(self, low, high, shape, dtype=np.float32):
        self.low, self.high, self.dtype = np.asarray(low), np.asarray(high), dtype
        self.shape = tuple(shape)


class Discrete:
    def __init__(self, n):
        self.n = n


def _spaces():
    # environment.py:51-62
    position_low = np.array([-500000, -500000, -500000, -10000000, -10000000, -10000000, -10000000, -10000000,
                             -10000000])
    velocity_low = np.array([-10000, -10000, -10000, -50000, -50000, -50000, -50000, -50000, -50000])
    low = np.concatenate((position_low, velocity_low))
    obs = Box(low=low, high=-low, shape=(OBS_DIM,), dtype=np.float32)
    act = np.array([[-1.6, 1.6], [-1.6, 1.6], [-1.6, 1.6]])
    return obs, act, Discrete(5)


class VecSatellites:
    """``num_envs`` reference environments stepped by one HIP kernel launch.

    Tensors are device tensors on ``device`` (actions f32 [N,3]); every call
    is asynchronous on the current torch stream.  device="cpu": the host
    build (satenv_cpu_*, synchronous, `threads` OpenMP threads, 0 = all)."""

    def __init__(self, num_envs: int, device=None, d_capture: float = 100000.0, d_range: float = 100000.0,
                 max_episode_steps: int = 1000, Flag: int = 0, fuel_c=320, fuel_t=320, threads: int = 0, **params):
        self.host = device is not None and torch.device(device).type == "cpu"
        if not self.host and not torch.cuda.is_available():
            raise _lib.NativeError("VecSatellites needs a HIP device (MI355X); the host build runs only when asked "
                                   "for with device='cpu'")
        if self.host:
            self.device = torch.device("cpu")
        else:
            self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self._api = "satenv_cpu_" if self.host else "satenv_"
        self._req = require_cpu if self.host else require_cuda
        self.num_envs = int(num_envs)
        self._p = default_params(d_capture=float(d_capture), d_range=float(d_range),
                                 max_episode_steps=int(max_episode_steps), flag=int(Flag), fuel_c0=float(fuel_c),
                                 fuel_t0=float(fuel_t), fuel_c0_mode=_num_mode(fuel_c),
                                 fuel_t0_mode=_num_mode(fuel_t), **params)
        h = C.c_void_p()
        if self.host:
            check(self._fn("create")(C.byref(h), self.num_envs, C.byref(self._p), int(threads)), "satenv_cpu_create")
        else:
            with torch.cuda.device(self.device):
                check(_lib.lib().satenv_create(C.byref(h), self.num_envs, C.byref(self._p), self.device.index or 0),
                      "satenv_create")
        self._h = h
        self.observation_space, self.action_space, self.action_space_beta = _spaces()
        self.stats = torch.zeros(4, dtype=torch.float64, device=self.device)

    def _fn(self, name):
        return getattr(_lib.lib(), self._api + name)

    def _sp(self):
        return None if self.host else stream_ptr()

    # -- parameters -----------------------------------------------------------
    def _push_params(self):
        check(self._fn("set_params")(self._h, C.byref(self._p)), self._api + "set_params")

    def set_params(self, **fields):
        """Update satenv_params fields (e.g. propagator=2) and push them."""
        for k, v in fields.items():
            if not hasattr(self._p, k):
                raise AttributeError(f"satenv_params has no field {k!r}")
            setattr(self._p, k, v)
        self._push_params()

    @property
    def d_capture(self):
        return self._p.d_capture

    @d_capture.setter
    def d_capture(self, v):          # CPPO_main.py:98 "env.d_capture = d_capture"
        self._p.d_capture = float(v)
        self._push_params()

    @property
    def max_episode_steps(self):
        return self._p.max_episode_steps

    @max_episode_steps.setter
    def max_episode_steps(self, v):
        self._p.max_episode_steps = int(v)
        self._push_params()

    @property
    def d_range(self):
        return self._p.d_range

    @d_range.setter
    def d_range(self, v):
        self._p.d_range = float(v)
        self._push_params()

    def set_step_kernel(self, kind: int = 2, wide_envs: int = 64):
        """Which step kernel the device build launches (satenv_set_step_kernel):
        2 the wide kernel (default), 1 the four-solve split kernel, 0 one lane
        per env; every one computes the same bits."""
        if self.host:
            raise _lib.NativeError("the host build has one step loop")
        check(_lib.lib().satenv_set_step_kernel(self._h, int(kind), int(wide_envs)), "satenv_set_step_kernel")

    # -- API -----------------------------------------------------------------
    def reset(self, Flag: int = 0, mask=None, obs_out=None, obs64_out=None):
        """environment.py:66-79 for all envs (or those with mask != 0). Returns obs f32 [N,18]."""
        n = self.num_envs
        if obs_out is None and obs64_out is None:
            obs_out = torch.empty((n, OBS_DIM), dtype=torch.float32, device=self.device)
        if mask is not None:
            self._req(mask, torch.uint8, (n,), "mask")
        check(self._fn("reset")(self._h, int(Flag), ptr(mask), ptr(obs_out), ptr(obs64_out), self._sp()),
              self._api + "reset")
        return obs_out if obs_out is not None else obs64_out

    def step(self, pursuer_action, escaper_action, epsiode_count=None, obs_out=None, obs64_out=None,
             reward_out=None, done_out=None):
        """environment.py:81-255 for all envs, no automatic reset.

        Returns (obs f32 [N,18] or obs64, reward f64 [N], done u8 [N])."""
        n = self.num_envs
        self._req(pursuer_action, torch.float32, (n, ACT_DIM), "pursuer_action")
        self._req(escaper_action, torch.float32, (n, ACT_DIM), "escaper_action")
        if epsiode_count is not None:
            self._req(epsiode_count, torch.int32, (n,), "epsiode_count")
        if obs_out is None and obs64_out is None:
            obs_out = torch.empty((n, OBS_DIM), dtype=torch.float32, device=self.device)
        if reward_out is None:
            reward_out = torch.empty(n, dtype=torch.float64, device=self.device)
        if done_out is None:
            done_out = torch.empty(n, dtype=torch.uint8, device=self.device)
        check(self._fn("step")(self._h, ptr(pursuer_action), ptr(escaper_action), ptr(epsiode_count), ptr(obs_out),
                               ptr(obs64_out), ptr(reward_out), ptr(done_out), self._sp()), self._api + "step")
        return (obs_out if obs_out is not None else obs64_out), reward_out, done_out

    def step_autoreset(self, pursuer_action, escaper_action, obs_out=None, reward_out=None, done_out=None,
                       stats=True):
        """One step of the CPPO_main.py:119-153 loop for all envs: device episode
        counters, done envs reset in-kernel (obs_out = post-reset obs).
        Returns (obs f32 [N,18], reward f32 [N], done u8 [N])."""
        n = self.num_envs
        if obs_out is None:
            obs_out = torch.empty((n, OBS_DIM), dtype=torch.float32, device=self.device)
        if reward_out is None:
            reward_out = torch.empty(n, dtype=torch.float32, device=self.device)
        if done_out is None:
            done_out = torch.empty(n, dtype=torch.uint8, device=self.device)
        if self.host:
            self._req(pursuer_action, torch.float32, (n, ACT_DIM), "pursuer_action")
            self._req(escaper_action, torch.float32, (n, ACT_DIM), "escaper_action")
        check(self._fn("step_autoreset")(self._h, ptr(pursuer_action), ptr(escaper_action), ptr(obs_out),
                                         ptr(reward_out), ptr(done_out), ptr(self.stats) if stats else None,
                                         self._sp()), self._api + "step_autoreset")
        return obs_out, reward_out, done_out

    def get_state(self):
        n = self.num_envs
        f = torch.empty((SATENV_F64_PLANES, n), dtype=torch.float64, device=self.device)
        i = torch.empty((SATENV_I32_PLANES, n), dtype=torch.int32, device=self.device)
        check(self._fn("get_state")(self._h, ptr(f), ptr(i), self._sp()), self._api + "get_state")
        return f, i

    def set_state(self, f64_planes=None, i32_planes=None):
        n = self.num_envs
        if f64_planes is not None:
            self._req(f64_planes, torch.float64, (SATENV_F64_PLANES, n), "f64_planes")
        if i32_planes is not None:
            self._req(i32_planes, torch.int32, (SATENV_I32_PLANES, n), "i32_planes")
        check(self._fn("set_state")(self._h, ptr(f64_planes), ptr(i32_planes), self._sp()), self._api + "set_state")

    def check_errors(self) -> int:
        st = C.c_int32(0)
        check(self._fn("check")(self._h, C.byref(st)), self._api + "check")
        return st.value

    def close(self):
        if getattr(self, "_h", None):
            self._fn("destroy")(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pack_bits(fuel_c_mode, fuel_t_mode, vel_int, flag):
    return (int(fuel_c_mode) & 3) | ((int(fuel_t_mode) & 3) << 2) | ((int(vel_int) & 1) << 4) | ((int(flag) & 3) << 5)


def unpack_bits(b):
    b = int(b)
    return dict(fuel_c_mode=b & 3, fuel_t_mode=(b >> 2) & 3, vel_int=(b >> 4) & 1, flag=(b >> 5) & 3)


def _typed(v, mode):
    return [int(v), np.int64(v), np.float32(v), np.float64(v)][mode]


class satellites:  # noqa: N801  (reference class name)
    """Drop-in for ``environment.satellites`` (environment.py:8), Flag 0/1/2.

    Same keywords as environment.py:26-28; ``args.max_episode_steps`` is
    required as in environment.py:46.  State lives on the GPU; the public
    attributes are read back on access.  Flag 2 (environment.py:257-315):
    the kernel steps the state (no danger-zone update, reward 0), the
    ellipse_params come from the reachable-domain grid and ellipse-fit
    kernels (satrl.reachable), and the env's network_method_train takes its
    step on the CPU like the reference's.
    """

    def __init__(self, Pursuer_position=np.array([2000, 2000, 1000]), Pursuer_vector=np.array([1.71, 1.14, 1.3]),
                 Escaper_position=np.array([1000, 2000, 0]), Escaper_vector=np.array([1.71, 1.14, 1.3]),
                 M=0.4, dis_safe=1000, d_capture=100000, Flag=0, fuel_c=320, fuel_t=320, d_range=100000,
                 args=None, device=None):
        max_ep = args.max_episode_steps          # AttributeError on args=None, as environment.py:46
        kin = np.concatenate([np.asarray(Pursuer_position, np.float64), np.asarray(Pursuer_vector, np.float64),
                              np.asarray(Escaper_position, np.float64), np.asarray(Escaper_vector, np.float64)])
        self._v = VecSatellites(1, device=device, d_capture=d_capture, d_range=d_range, max_episode_steps=max_ep,
                                Flag=Flag, fuel_c=fuel_c, fuel_t=fuel_t, init_kin=kin)
        self.dis_dafe = dis_safe
        self.M = M
        self.burn_reward = 0
        self.win_reward = 100
        self.ellipse_params = []
        self.observation_space, self.action_space, self.action_space_beta = _spaces()
        # environment.py:49 builds the ellipse-fitting trainer, whose ImprovedNN()
        # (real_time_data_process.py:129) draws its default init from torch's
        # global CPU generator: draw the same numbers, so agents constructed
        # after a seeded env get the reference's weights
        from .surrogate import network_method_train
        self.trian_elliptical_fitting = network_method_train(pretrain=False,
                                                             save_dir=getattr(args, "ellipse_save_dir", None))
        dev = self._v.device
        self._pa = torch.empty((1, ACT_DIM), dtype=torch.float32, device=dev)
        self._ea = torch.empty((1, ACT_DIM), dtype=torch.float32, device=dev)
        self._cnt = torch.empty(1, dtype=torch.int32, device=dev)
        self._obs = torch.empty((1, OBS_DIM), dtype=torch.float64, device=dev)
        self._r = torch.empty(1, dtype=torch.float64, device=dev)
        self._d = torch.empty(1, dtype=torch.uint8, device=dev)

    # reference attributes ------------------------------------------------------
    d_capture = property(lambda s: s._v.d_capture, lambda s, v: setattr(s._v, "d_capture", v))
    d_range = property(lambda s: s._v.d_range, lambda s, v: setattr(s._v, "d_range", v))
    max_episode_steps = property(lambda s: s._v.max_episode_steps,
                                 lambda s, v: setattr(s._v, "max_episode_steps", v))

    def _state(self):
        f, i = self._v.get_state()
        return f[:, 0].cpu().numpy(), i[:, 0].cpu().numpy()

    def _set(self, fi=None, ii=None):
        f, i = self._v.get_state()
        if fi:
            for k, v in fi.items():
                f[k, 0] = v
        if ii:
            for k, v in ii.items():
                i[k, 0] = v
        self._v.set_state(f, i)

    def _kin(self, lo):
        f, i = self._state()
        vel_int = unpack_bits(i[2])["vel_int"]
        arr = f[lo:lo + 3].copy()
        return arr.astype(np.int64) if vel_int else arr

    Pursuer_position = property(lambda s: s._kin(0))
    Pursuer_vector = property(lambda s: s._kin(3))
    Escaper_position = property(lambda s: s._kin(6))
    Escaper_vector = property(lambda s: s._kin(9))

    @property
    def fuel_c(self):
        f, i = self._state()
        return _typed(f[12], unpack_bits(i[2])["fuel_c_mode"])

    @fuel_c.setter
    def fuel_c(self, v):
        f, i = self._v.get_state()
        b = unpack_bits(int(i[2, 0]))
        f[12, 0] = float(v)
        i[2, 0] = pack_bits(_num_mode(v), b["fuel_t_mode"], b["vel_int"], b["flag"])
        self._v.set_state(f, i)

    @property
    def fuel_t(self):
        f, i = self._state()
        return _typed(f[13], unpack_bits(i[2])["fuel_t_mode"])

    @property
    def dis(self):
        return float(self._state()[0][14])

    @property
    def dangerous_zone(self):
        return int(self._state()[1][0])

    @property
    def Flag(self):
        return unpack_bits(self._state()[1][2])["flag"]

    # API ------------------------------------------------------------------------
    def reset(self, Flag):
        """environment.py:66-79: returns the int64 observation."""
        if Flag not in (0, 1, 2):
            raise ValueError(f"Flag must be 0, 1 or 2 (environment.py:36), got {Flag!r}")
        self._v.reset(Flag, obs64_out=self._obs)
        return self._obs[0].cpu().numpy().astype(np.int64)

    def step(self, pursuer_action, escaper_action, epsiode_count):
        """environment.py:81-255.  Actions are taken as float32 (the dtype
        PPO_continuous.choose_action returns)."""
        self._pa.copy_(torch.as_tensor(np.asarray(pursuer_action, dtype=np.float32).reshape(1, ACT_DIM)))
        self._ea.copy_(torch.as_tensor(np.asarray(escaper_action, dtype=np.float32).reshape(1, ACT_DIM)))
        self._cnt.fill_(int(epsiode_count))
        self._v.step(self._pa, self._ea, self._cnt, obs_out=None, obs64_out=self._obs, reward_out=self._r,
                     done_out=self._d)
        obs = self._obs[0].cpu().numpy().copy()      # a fresh array per step (on device="cpu" .cpu() aliases)
        r = float(self._r.item())
        done = bool(self._d.item())
        if done:
            r = int(r)          # terminal rewards are python ints in the reference
        if self.Flag == 2:
            self._flag2_fit()
            r = 0               # environment.py:298-315 return the literal 0
        return obs, r, done

    def _flag2_fit(self):
        """environment.py:293-301: ellipse_params = numerical_method_process(
        R0_c, V0_c, fuel_c) on the GPU grid + fit kernels, then one step of
        the env's ellipse-fitting network."""
        from . import reachable as RD
        if self._v.host:
            raise _lib.NativeError("Flag 2's reachable-domain grid and ellipse fit run on the GPU kernels; the host "
                                   "build steps Flag 0/1 only")
        orbits, status = RD.env_orbits(self._v)
        if int(status.item()) != 0:
            # real_time_data_process.py:109 -> RD_single_pulse.py:32 indexes data[5] of a 4/5-element list
            raise IndexError("list index out of range (the pursuer's orbit has no 6-element set, "
                             f"satenv code {int(status.item())})")
        ell, _ = RD.reachable_ellipses(orbits, RD.params["N1"], RD.params["N2"], RD.params["N3"])
        self.ellipse_params = ell[0].cpu().numpy()
        R0_c, V0_c = self.relative_state_to_absolute_state(self.Pursuer_position, self.Pursuer_vector)
        self.trian_elliptical_fitting.train(R0_c, V0_c, self.fuel_c, self.ellipse_params)

    @staticmethod
    def relative_state_to_absolute_state(R0, V0):
        """environment.py:334-343."""
        assert isinstance(R0, np.ndarray) and isinstance(V0, np.ndarray)
        return np.array([27098000, 32306000, 0]) + R0, np.array([-2350, 1970, 0]) + V0
