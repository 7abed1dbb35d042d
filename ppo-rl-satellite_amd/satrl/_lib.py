"""ctypes binding of the product's C-ABI library ``libsatrl.so``.

The library exports exactly the functions declared in ``include/satenv.h``
and ``include/satrl_rollout.h`` (plain pointers, sizes and a ``void*``
hipStream_t).  It is built in-tree by ``csrc/Makefile`` for gfx950.  There is
no fallback: if the library is missing or cannot be loaded, every op raises.

torch is imported first so that the process has a single HIP runtime
(torch's bundled ``libamdhip64.so.7``; the library's NEEDED entry resolves to
it by SONAME).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import torch  # noqa: F401  (must be loaded before libsatrl.so, see module doc)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC_DIR = os.path.join(os.path.dirname(PKG_DIR), "csrc")
LIB_PATH = _PRODUCT_LIB = os.path.join(PKG_DIR, "libsatrl.so")
# development A/B builds only (tools/_probe variants); the shipped path is LIB_PATH
LIB_PATH = os.environ.get("SATRL_LIB_PATH", LIB_PATH)

SATENV_F64_PLANES = 15
SATENV_I32_PLANES = 3
OBS_DIM = 18
ACT_DIM = 3


class SatenvParams(C.Structure):
    """Mirror of ``satenv_params`` (include/satenv.h)."""
    _fields_ = [("d_capture", C.c_double), ("d_range", C.c_double), ("win_reward", C.c_double),
                ("burn_reward", C.c_double), ("mu", C.c_double), ("R_cw", C.c_double * 3),
                ("V_cw", C.c_double * 3), ("stm", C.c_double * 36), ("fuel_c0", C.c_double),
                ("fuel_t0", C.c_double), ("init_kin", C.c_double * 12), ("max_episode_steps", C.c_int32),
                ("flag", C.c_int32), ("fuel_c0_mode", C.c_int32), ("fuel_t0_mode", C.c_int32),
                ("cw_omega", C.c_double), ("propagator", C.c_int32), ("rk4_substeps", C.c_int32)]


class NativeError(RuntimeError):
    pass


def build(force: bool = False) -> str:
    """Compile libsatrl.so for gfx950 with hipcc (csrc/Makefile)."""
    args = ["make", "-s", "-C", CSRC_DIR, "-j4"]
    if force:
        subprocess.check_call(["make", "-s", "-C", CSRC_DIR, "clean"])
    subprocess.check_call(args)
    return LIB_PATH


_lib = None

_vp = C.c_void_p
_i64 = C.c_int64
_i32 = C.c_int32
_SIGS = {
    "satenv_default_params": ([C.POINTER(SatenvParams)], C.c_int),
    "satenv_stm": ([C.c_double, C.POINTER(C.c_double)], C.c_int),
    "satenv_last_error": ([], C.c_char_p),
    "satenv_abi_version": ([], C.c_int),
    "satenv_create": ([C.POINTER(_vp), _i64, C.POINTER(SatenvParams), C.c_int], C.c_int),
    "satenv_destroy": ([_vp], C.c_int),
    "satenv_num_envs": ([_vp, C.POINTER(_i64)], C.c_int),
    "satenv_set_params": ([_vp, C.POINTER(SatenvParams)], C.c_int),
    "satenv_set_step_kernel": ([_vp, C.c_int32, C.c_int32], C.c_int),
    "satenv_reset": ([_vp, _i32, _vp, _vp, _vp, _vp], C.c_int),
    "satenv_step": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "satenv_step_autoreset": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "satenv_get_state": ([_vp, _vp, _vp, _vp], C.c_int),
    "satenv_set_state": ([_vp, _vp, _vp, _vp], C.c_int),
    "satenv_check": ([_vp, C.POINTER(_i32)], C.c_int),
    "satenv_danger_zone": ([_i64, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "satenv_solve_alpha": ([_i64, _vp, _vp, _vp], C.c_int),
    "satenv_sincos": ([_i64, _vp, _vp, _vp, _i32, _vp], C.c_int),
    "satenv_acos": ([_i64, _vp, _vp, _i32, _vp], C.c_int),
    "satenv_rk4_j2": ([_i64, _vp, C.c_double, _i32, _vp, _vp], C.c_int),
    "satenv_reachable_domain": ([_i64, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp], C.c_int),
    "satenv_surrogate_blob_bytes": ([], C.c_int),
    "satenv_surrogate_pack": ([_vp] * 10, C.c_int),
    "satenv_surrogate": ([_vp, _vp, _vp, _vp], C.c_int),
    "satenv_surrogate_mlp": ([_i64, _vp, _vp, _vp, _vp], C.c_int),
    "satenv_surrogate_set_scalers": ([_vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "satenv_ellipse_fit": ([_i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "satenv_rd_orbits": ([_vp, _vp, _vp, _vp], C.c_int),
    "satenv_cpu_last_error": ([], C.c_char_p),
    "satenv_cpu_create": ([C.POINTER(_vp), _i64, C.POINTER(SatenvParams), C.c_int], C.c_int),
    "satenv_cpu_destroy": ([_vp], C.c_int),
    "satenv_cpu_num_envs": ([_vp, C.POINTER(_i64)], C.c_int),
    "satenv_cpu_set_params": ([_vp, C.POINTER(SatenvParams)], C.c_int),
    "satenv_cpu_reset": ([_vp, _i32, _vp, _vp, _vp, _vp], C.c_int),
    "satenv_cpu_step": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "satenv_cpu_step_autoreset": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "satenv_cpu_get_state": ([_vp, _vp, _vp, _vp], C.c_int),
    "satenv_cpu_set_state": ([_vp, _vp, _vp, _vp], C.c_int),
    "satenv_cpu_danger_zone": ([_i64, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "satenv_cpu_check": ([_vp, C.POINTER(_i32)], C.c_int),
    "satrl_gae": ([_i64, _i64, _vp, _vp, _vp, C.c_float, C.c_float, _vp, _vp, _vp], C.c_int),
    "satrl_gaussian_sample": ([_i64, _vp, _vp, C.c_float, C.c_uint64, C.c_uint32, _i64, C.c_uint64, _vp, _vp, _vp,
                               _vp],
                              C.c_int),
    "satrl_moments": ([_i64, _vp, _vp, _vp], C.c_int),
    "satrl_last_error": ([], C.c_char_p),
    "satrl_ppo_layout": ([C.c_int, C.POINTER(_i64)], C.c_int),
    "satrl_ppo_sizes": ([C.c_int, C.c_int, C.POINTER(_i64), C.POINTER(_i64)], C.c_int),
    "satrl_ppo_dw2_splits": ([C.c_int, C.c_int], C.c_int),
    "satrl_ppo_dw2": ([C.c_int, C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _i64, _vp], C.c_int),
    "satrl_ppo_reduce": ([C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp],
                         C.c_int),
    "satrl_ppo_reduce_dp": ([C.c_int, C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    "satrl_ppo_adam": ([C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, C.c_int, _vp, C.c_float, C.c_float, C.c_float,
                        C.c_float, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "satrl_ppo_rowpass": ([C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _vp, C.c_float, C.c_float, C.c_float, _vp, _vp,
                           _vp, _vp, _vp], C.c_int),
    "satrl_ppo_rowpass_ratio": ([C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _vp, C.c_float, C.c_float, C.c_float, _vp,
                                 _vp, _vp, _vp, _vp, _vp], C.c_int),
    "satrl_ppo_row_blocks": ([C.c_int, C.c_int], C.c_int),
    "satrl_ppo_w2x_floats": ([C.c_int], _i64),
    "satrl_ppo_kx_elems": ([C.c_int, C.c_int], _i64),
    "satrl_ppo_rowpass_kx": ([C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _vp, C.c_float, C.c_float, C.c_float, _vp,
                              _vp, _i64, _vp, _vp, _vp], C.c_int),
    "satrl_ppo_dw2_kx_splits": ([C.c_int, C.c_int, C.c_int], C.c_int),
    "satrl_ppo_rowpass_error": ([C.POINTER(C.c_int), C.c_double, _vp], C.c_int),
    "satrl_ppo_rowpass_fault_inject": ([C.c_int, C.c_uint, _vp], C.c_int),
    "satrl_ppo_dw2_kx": ([C.c_int, C.c_int, C.c_int, C.c_int, _vp, _vp, _i64, _vp, _i64, _vp], C.c_int),
    "satrl_ppo_dw2_kx_w1": ([C.c_int, C.c_int, C.c_int, C.c_int, _vp, _vp, _i64, _vp, _i64, C.c_int, _vp, _vp, _vp,
                             _vp, _vp], C.c_int),
    "satrl_ppo_w2x_sync": ([C.c_int, C.c_int, _vp, _vp, _vp], C.c_int),
    "satrl_ppo_rowpass_dw2": ([C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _vp, C.c_float, C.c_float, C.c_float, _vp,
                               _i64, _vp, _vp, _vp], C.c_int),
    "satrl_peer_buffer_bytes": ([_i64, C.c_int, _vp], C.c_int),
    "satrl_peer_alloc": ([_i64, _vp, _vp], C.c_int),
    "satrl_peer_open": ([_vp, _vp], C.c_int),
    "satrl_peer_close": ([_vp], C.c_int),
    "satrl_peer_free": ([_vp], C.c_int),
    "satrl_peer_error": ([_vp, _vp, _vp], C.c_int),
    "satrl_peer_reset": ([_vp, _i64, _vp], C.c_int),
    "satrl_peer_blocks": ([C.c_int, _vp], C.c_int),
    "satrl_ppo_allreduce_peer": ([C.c_int, C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _vp, C.c_int, C.c_double,
                                  _vp], C.c_int),
    "satrl_policy_act": ([C.c_int, _i64, _vp, _vp, _vp, C.c_float, C.c_uint64, _i64, C.c_uint64, _vp, _vp, _vp, _vp,
                          _vp, _vp], C.c_int),
    "satrl_policy_value": ([C.c_int, _i64, _vp, _vp, _vp, _vp], C.c_int),
    "satrl_ppo_stage": ([_i64, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "satrl_ppo_group_advance": ([_vp, _vp], C.c_int),
    "satrl_ppo_tanh": ([_i64, _vp, _vp, _vp], C.c_int),
    "satrl_span_probe": ([_vp, _i64, _vp], C.c_int),
    "satrl_span_probe_launches": ([], _i64),
    "satrl_span_probe_launch": ([_i64, _vp, _vp, _vp], C.c_int),
    "satrl_ppo_last_error": ([], C.c_char_p),
}


def exported_symbols():
    return sorted(_SIGS)


def lib():
    """Load libsatrl.so (raises NativeError if it is absent/unloadable)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"{LIB_PATH} not built: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
        try:
            L = C.CDLL(LIB_PATH)
        except OSError as e:
            raise NativeError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (argt, rest) in _SIGS.items():
            if LIB_PATH != _PRODUCT_LIB and not hasattr(L, name):
                continue                     # (an older development build: A/B only)
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = rest
        _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        L = lib()
        msg = (L.satenv_cpu_last_error() if what.startswith("satenv_cpu") else
               L.satenv_last_error() if what.startswith("satenv") else
               L.satrl_ppo_last_error() if what.startswith(("satrl_ppo", "satrl_peer")) else
               L.satrl_last_error()).decode()
        raise NativeError(f"{what} failed ({rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = torch.cuda.current_stream() if stream is None else stream
    return C.c_void_p(s.cuda_stream)


def require_cpu(t, dtype, shape=None, name="tensor"):
    """Host-build (satenv_cpu_*) argument check: a contiguous CPU tensor."""
    if t.is_cuda:
        raise NativeError(f"{name} must be a host (cpu) tensor for the host build")
    return _require(t, dtype, shape, name)


def require_cuda(t, dtype, shape=None, name="tensor"):
    if not t.is_cuda:
        raise NativeError(f"{name} must be a device (cuda/HIP) tensor")
    return _require(t, dtype, shape, name)


def _require(t, dtype, shape, name):
    if t.dtype != dtype:
        raise NativeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise NativeError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise NativeError(f"{name} shape {tuple(t.shape)} != {tuple(shape)}")
    return t
