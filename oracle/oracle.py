"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes front-end of the plain-C restatement (``satenv_oracle.c``) plus numpy /
torch-CPU restatements of the learning-side hot path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module; the product package never does (and fails loudly without its HIP
library instead of falling back here).

Reference citations are ``file:line`` in qiaobeibei/PPO-RL-Satellite.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle_satenv.so")

PYINT, I64, F32, F64 = 0, 1, 2, 3


class OrcEnv(C.Structure):
    _fields_ = [("Pp", C.c_double * 3), ("Pv", C.c_double * 3), ("Ep", C.c_double * 3),
                ("Ev", C.c_double * 3), ("fuel_c", C.c_double), ("fuel_t", C.c_double),
                ("dis", C.c_double), ("dz", C.c_int32), ("fuel_c_mode", C.c_int32),
                ("fuel_t_mode", C.c_int32), ("vel_int", C.c_int32), ("flag", C.c_int32)]


class OrcParams(C.Structure):
    _fields_ = [("d_capture", C.c_double), ("d_range", C.c_double), ("win_reward", C.c_double),
                ("burn_reward", C.c_double), ("max_episode_steps", C.c_int32), ("mu", C.c_double),
                ("R_cw", C.c_double * 3), ("V_cw", C.c_double * 3), ("stm", C.c_double * 36),
                ("cw_omega", C.c_double), ("propagator", C.c_int32), ("rk4_substeps", C.c_int32)]


def build() -> str:
    """Compile the oracle with its Makefile (gcc); returns the .so path."""
    subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        dp = C.POINTER(C.c_double)
        fp = C.POINTER(C.c_float)
        ip = C.POINTER(C.c_int32)
        L.orc_default_params.argtypes = [C.POINTER(OrcParams), C.c_double, C.c_int32]
        L.orc_stm.argtypes = [C.c_double, dp]
        L.orc_env_init.argtypes = [C.POINTER(OrcEnv)]
        L.orc_reset.argtypes = [C.POINTER(OrcEnv), C.c_int32, dp]
        L.orc_step.argtypes = [C.POINTER(OrcParams), C.POINTER(OrcEnv), fp, fp, C.c_int32, dp, dp, ip]
        L.orc_step.restype = C.c_int
        L.orc_danger_zone.argtypes = [dp, dp, dp, dp, C.c_double, C.c_int32, ip]
        L.orc_danger_zone.restype = C.c_int
        L.orc_orbital_elements.argtypes = [C.c_double, dp, dp, dp]
        L.orc_orbital_elements.restype = C.c_int
        L.orc_solve_alpha.argtypes = [C.c_double] * 7 + [ip]
        L.orc_solve_alpha.restype = C.c_double
        L.orc_set_jitter.argtypes = [C.c_ulonglong]
        L.orc_step_planes.argtypes = [C.POINTER(OrcParams), C.c_int64, dp, ip, fp, fp, ip, dp, ip, C.c_int32]
        L.orc_step_planes.restype = C.c_int
        L.orc_rollout.argtypes = [C.POINTER(OrcParams), C.POINTER(OrcEnv), C.c_int64, C.c_int32,
                                  fp, fp, ip, dp, ip, C.c_int32]
        L.orc_rollout.restype = C.c_int
        L.orc_rk4_j2_rhs.argtypes = [dp, dp]
        L.orc_rk4_j2_step.argtypes = [dp, C.c_double, dp]
        L.orc_rk4_j2_propagate.argtypes = [dp, C.c_double, C.c_int32]
        L.orc_cw_rk4.argtypes = [dp, C.c_double, C.c_double, C.c_int32, dp]
        L.orc_cw_rk45.argtypes = [dp, C.c_double, dp, ip]
        L.orc_cw_rk45.restype = C.c_int32
        L.orc_reachable_domain.argtypes = [C.POINTER(OrcRdParams), dp, dp, C.POINTER(C.c_uint8)]
        L.orc_reachable_domain.restype = C.c_int64
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def params(d_capture=15000.0, max_episode_steps=1000, d_range=100000.0, propagator=0, rk4_substeps=10):
    p = OrcParams()
    lib().orc_default_params(C.byref(p), float(d_capture), int(max_episode_steps))
    p.d_range = float(d_range)
    p.propagator = int(propagator)
    p.rk4_substeps = int(rk4_substeps)
    return p


def rk4_j2(rv0, h, steps):
    """轨道外推-龙格库塔算法.py RungeKutta applied `steps` times, batched [n][6]."""
    rv = np.array(rv0, dtype=np.float64, copy=True).reshape(-1, 6)
    for row in rv:
        buf = np.ascontiguousarray(row)
        lib().orc_rk4_j2_propagate(_dp(buf), float(h), int(steps))
        row[:] = buf
    return rv


def rk4_j2_rhs(rv):
    out = np.zeros(6)
    lib().orc_rk4_j2_rhs(_dp(np.ascontiguousarray(rv, dtype=np.float64)), _dp(out))
    return out


def cw_rk4(x, w, t, nsub):
    y = np.zeros(6)
    lib().orc_cw_rk4(_dp(np.ascontiguousarray(x, dtype=np.float64)), float(w), float(t), int(nsub), _dp(y))
    return y


def cw_rk45(x, t):
    """Numerical_calculation_method.numerical_calculation(t) of one craft
    (satellite_function.py:783-839): (state after t seconds, nfev)."""
    y = np.zeros(6)
    nfev = np.zeros(1, dtype=np.int32)
    rc = lib().orc_cw_rk45(_dp(np.ascontiguousarray(x, dtype=np.float64)), float(t), _dp(y),
                           nfev.ctypes.data_as(C.POINTER(C.c_int32)))
    if rc:
        raise ValueError(f"orc_cw_rk45: {rc}")
    return y, int(nfev[0])


def stm(t=100.0):
    out = np.zeros(36)
    lib().orc_stm(float(t), _dp(out))
    return out.reshape(6, 6)


class OrcRdParams(C.Structure):
    _fields_ = [("a", C.c_double), ("e0", C.c_double), ("f", C.c_double), ("delta_max", C.c_double),
                ("mu", C.c_double), ("n1", C.c_int32), ("n2", C.c_int32), ("n3", C.c_int32),
                ("dv_f32", C.c_int32)]


def reachable_domain_grid(a, e0, f, delta_max, n1=1, n2=200, n3=200, mu=3.986e14, dv_f32=False):
    """RD_single_pulse.py:40-148 over the whole direction grid: returns
    (rf_max [n][3], rf_min [n][3], status [n] u8) with n = n1*(n2+1)*(n3+1).
    dv_f32: delta_max is an np.float32 scalar (Delta_V in float32)."""
    p = OrcRdParams(float(a), float(e0), float(f), float(delta_max), float(mu), int(n1), int(n2), int(n3),
                    int(bool(dv_f32)))
    n = int(n1) * (int(n2) + 1) * (int(n3) + 1)
    mx = np.zeros((n, 3))
    mn = np.zeros((n, 3))
    st = np.zeros(n, dtype=np.uint8)
    lib().orc_reachable_domain(C.byref(p), _dp(mx), _dp(mn), st.ctypes.data_as(C.POINTER(C.c_uint8)))
    return mx, mn, st


def reachable_domain(a, e0, f, delta_max, n1=1, n2=200, n3=200, mu=3.986e14, dv_f32=False):
    """The RF_max / RF_min point lists Reachable_Domain hands to Curve_fitting
    (RD_single_pulse.py:138-140), in the reference's loop order."""
    mx, mn, st = reachable_domain_grid(a, e0, f, delta_max, n1, n2, n3, mu, dv_f32)
    if (st == 2).any():
        raise ValueError("gama - f outside the theta branches of RD_single_pulse.py:87-90")
    keep = st == 1
    return mx[keep], mn[keep]


def solve_alpha(u, dvm, theta, v1x, v1y, h, guess):
    nfev = C.c_int32(0)
    x = lib().orc_solve_alpha(u, dvm, theta, v1x, v1y, h, guess, C.byref(nfev))
    return x, nfev.value


def orbital_elements(R, V, mu=3.986e14):
    R = np.ascontiguousarray(R, dtype=np.float64)
    V = np.ascontiguousarray(V, dtype=np.float64)
    out = np.zeros(6)
    rc = lib().orc_orbital_elements(mu, _dp(R), _dp(V), _dp(out))
    return rc, out


def danger_zone(Rc, Vc, Rt, Vt, fuel, fuel_mode):
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (Rc, Vc, Rt, Vt)]
    cnt = C.c_int32(0)
    rc = lib().orc_danger_zone(*[_dp(a) for a in arrs], float(fuel), int(fuel_mode), C.byref(cnt))
    return rc, cnt.value


def set_jitter(seed):
    """libm-tie probe: seed != 0 moves transcendental results of the
    restatement by an ulp or two (satenv_oracle.c orc_jit); 0 = exact."""
    lib().orc_set_jitter(int(seed))


def dz_libm_tie(Rc, Vc, Rt, Vt, fuel, fuel_mode, target, seeds=2048):
    """Is danger-zone count `target` one ulp of libm away?  Returns the first
    jitter seed under which the restatement's count equals `target`, or 0
    if none of `seeds` seeds does (a count no ulp-level libm difference can
    explain)."""
    try:
        for s in range(1, int(seeds) + 1):
            set_jitter(s)
            rc, c = danger_zone(Rc, Vc, Rt, Vt, fuel, fuel_mode)
            if rc == 0 and c == int(target):
                return s
        return 0
    finally:
        set_jitter(0)


def step_planes(f64, i32, pa, ea, episode_count, d_capture=15000.0, max_episode_steps=1000, nthreads=8,
                propagator=0, rk4_substeps=10):
    """One step of n envs from SoA state planes (satenv_get_state layout:
    f64 [15][n], i32 [3][n]), no autoreset.  Returns (post f64, post i32,
    reward f64 [n], done i32 [n])."""
    p = params(d_capture, max_episode_steps, propagator=propagator, rk4_substeps=rk4_substeps)
    f = np.array(f64, dtype=np.float64, copy=True, order="C")
    i = np.array(i32, dtype=np.int32, copy=True, order="C")
    n = f.shape[1]
    pa = np.ascontiguousarray(pa, dtype=np.float32)
    ea = np.ascontiguousarray(ea, dtype=np.float32)
    cnt = np.ascontiguousarray(episode_count, dtype=np.int32)
    rew = np.zeros(n)
    done = np.zeros(n, dtype=np.int32)
    ip = C.POINTER(C.c_int32)
    rc = lib().orc_step_planes(C.byref(p), n, _dp(f), i.ctypes.data_as(ip), pa.ctypes.data_as(C.POINTER(C.c_float)),
                               ea.ctypes.data_as(C.POINTER(C.c_float)), cnt.ctypes.data_as(ip), _dp(rew),
                               done.ctypes.data_as(ip), int(nthreads))
    if rc != 0:
        raise RuntimeError("oracle step error")
    return f, i, rew, done


class OracleEnv:
    """N=1 environment on the C restatement (environment.py:8-343 semantics)."""

    def __init__(self, d_capture=15000.0, max_episode_steps=1000, d_range=100000.0, propagator=0, rk4_substeps=10):
        self.p = params(d_capture, max_episode_steps, d_range, propagator=propagator, rk4_substeps=rk4_substeps)
        self.e = OrcEnv()
        lib().orc_env_init(C.byref(self.e))

    def reset(self, flag=0):
        obs = np.zeros(18)
        lib().orc_reset(C.byref(self.e), int(flag), _dp(obs))
        return obs

    def step(self, pa, ea, episode_count):
        pa = np.ascontiguousarray(pa, dtype=np.float32)
        ea = np.ascontiguousarray(ea, dtype=np.float32)
        obs = np.zeros(18)
        r = C.c_double(0)
        d = C.c_int32(0)
        rc = lib().orc_step(C.byref(self.p), C.byref(self.e), pa.ctypes.data_as(C.POINTER(C.c_float)),
                            ea.ctypes.data_as(C.POINTER(C.c_float)), int(episode_count), _dp(obs),
                            C.byref(r), C.byref(d))
        if rc != 0:
            raise RuntimeError(f"oracle step error {rc}")
        return obs, r.value, bool(d.value)

    def get_state(self):
        e = self.e
        return dict(Pp=np.array(e.Pp[:]), Pv=np.array(e.Pv[:]), Ep=np.array(e.Ep[:]), Ev=np.array(e.Ev[:]),
                    fuel_c=e.fuel_c, fuel_t=e.fuel_t, dis=e.dis, dz=e.dz, fuel_c_mode=e.fuel_c_mode,
                    fuel_t_mode=e.fuel_t_mode, vel_int=e.vel_int, flag=e.flag)

    def set_state(self, st):
        e = self.e
        for k in ("Pp", "Pv", "Ep", "Ev"):
            getattr(e, k)[:] = [float(v) for v in st[k]]
        for k in ("fuel_c", "fuel_t", "dis"):
            setattr(e, k, float(st[k]))
        for k in ("dz", "fuel_c_mode", "fuel_t_mode", "vel_int", "flag"):
            setattr(e, k, int(st[k]))


def rollout(n_envs, steps, pa, ea, d_capture=15000.0, max_episode_steps=1000, nthreads=1, flag=0, propagator=0,
            rk4_substeps=10):
    """Batched replay from reset (CPU baseline).  pa/ea: float32 [steps, n, 3]."""
    p = params(d_capture, max_episode_steps, propagator=propagator, rk4_substeps=rk4_substeps)
    envs = (OrcEnv * n_envs)()
    for i in range(n_envs):
        lib().orc_env_init(C.byref(envs[i]))
        lib().orc_reset(C.byref(envs[i]), flag, None)
    cnt = np.zeros(n_envs, dtype=np.int32)
    rew = np.zeros((steps, n_envs))
    done = np.zeros((steps, n_envs), dtype=np.int32)
    pa = np.ascontiguousarray(pa, dtype=np.float32)
    ea = np.ascontiguousarray(ea, dtype=np.float32)
    rc = lib().orc_rollout(C.byref(p), envs, n_envs, steps, pa.ctypes.data_as(C.POINTER(C.c_float)),
                           ea.ctypes.data_as(C.POINTER(C.c_float)),
                           cnt.ctypes.data_as(C.POINTER(C.c_int32)), _dp(rew),
                           done.ctypes.data_as(C.POINTER(C.c_int32)), int(nthreads))
    if rc != 0:
        raise RuntimeError("oracle rollout error")
    return rew, done


class Rollout:
    """Like rollout() but the envs persist across run() calls (autoreset at
    done), so a long CPU sample can be fed in bounded action chunks."""

    def __init__(self, n_envs, d_capture=15000.0, max_episode_steps=1000, flag=0):
        self.n = int(n_envs)
        self.p = params(d_capture, max_episode_steps)
        self.envs = (OrcEnv * self.n)()
        for i in range(self.n):
            lib().orc_env_init(C.byref(self.envs[i]))
            lib().orc_reset(C.byref(self.envs[i]), flag, None)
        self.cnt = np.zeros(self.n, dtype=np.int32)

    def run(self, pa, ea, nthreads=1):
        steps = pa.shape[0]
        rew = np.zeros((steps, self.n))
        done = np.zeros((steps, self.n), dtype=np.int32)
        pa = np.ascontiguousarray(pa, dtype=np.float32)
        ea = np.ascontiguousarray(ea, dtype=np.float32)
        rc = lib().orc_rollout(C.byref(self.p), self.envs, self.n, steps, pa.ctypes.data_as(C.POINTER(C.c_float)),
                               ea.ctypes.data_as(C.POINTER(C.c_float)),
                               self.cnt.ctypes.data_as(C.POINTER(C.c_int32)), _dp(rew),
                               done.ctypes.data_as(C.POINTER(C.c_int32)), int(nthreads))
        if rc != 0:
            raise RuntimeError("oracle rollout error")
        return rew, done


# --------------------------------------------------------------------------
# Learning-side restatements (ppo_continuous.py)
# --------------------------------------------------------------------------
def gae_flat(r, vs, vs_, dw, done, gamma=0.99, lamda=0.95):
    """ppo_continuous.py:198-210 on one flat buffer (float32 like the reference)."""
    r = np.asarray(r, np.float32).reshape(-1)
    vs = np.asarray(vs, np.float32).reshape(-1)
    vs_ = np.asarray(vs_, np.float32).reshape(-1)
    dw = np.asarray(dw, np.float32).reshape(-1)
    done = np.asarray(done, np.float32).reshape(-1)
    # torch f32: r + (g*(1-dw))*vs_ - vs, python scalars rounded to f32
    deltas = ((r + (np.float32(gamma) * (np.float32(1.0) - dw)) * vs_) - vs).astype(np.float32)
    adv = np.zeros_like(deltas)
    # gamma*lamda is a python float; times an np.float32 it rounds to f32 (NEP 50)
    c = np.float32(gamma * lamda)
    gae = np.float32(0.0)
    for t in range(len(deltas) - 1, -1, -1):
        gae = np.float32(deltas[t] + np.float32(np.float32(c * gae) * np.float32(np.float32(1.0) - done[t])))
        adv[t] = gae
    return adv


def gae_time_major(r, vs, vs_, dw, done, gamma=0.99, lamda=0.95):
    """Per-env reverse scan over T of [T, N] arrays; each column is one flat
    reference buffer (ppo_continuous.py:204-206)."""
    T, N = np.shape(r)
    out = np.zeros((T, N), np.float32)
    for i in range(N):
        out[:, i] = gae_flat(r[:, i], vs[:, i], vs_[:, i], dw[:, i], done[:, i], gamma, lamda)
    return out


def gae_time_major_vec(r, vs, vs_, dw, done, gamma=0.99, lamda=0.95):
    """gae_time_major with the scan vectorised across envs: the same f32
    operations in the same order per element (numpy rounds every f32 array
    operation as it rounds the scalar ones), so it equals the per-env loop
    bit for bit (tests/test_oracle_golden.py pins that) at BASELINE sizes
    (T 2048 x N 16384) in seconds."""
    r = np.asarray(r, np.float32)
    vs = np.asarray(vs, np.float32)
    vs_ = np.asarray(vs_, np.float32)
    dw = np.asarray(dw, np.float32)
    done = np.asarray(done, np.float32)
    deltas = ((r + (np.float32(gamma) * (np.float32(1.0) - dw)) * vs_) - vs).astype(np.float32)
    c = np.float32(gamma * lamda)
    adv = np.zeros_like(deltas)
    gae = np.zeros(deltas.shape[1], np.float32)
    for t in range(deltas.shape[0] - 1, -1, -1):
        gae = (deltas[t] + (c * gae).astype(np.float32) * (np.float32(1.0) - done[t])).astype(np.float32)
        adv[t] = gae
    return adv
