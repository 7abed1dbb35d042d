"""satrl -- MI355X-native vectorised satellite pursuit-evasion PPO engine.

Hot path of qiaobeibei/PPO-RL-Satellite rebuilt for gfx950:
  * env step/reset: hand-written FP64 HIP kernel, one lane per env
    (csrc/satenv_kernels.hip, C-ABI include/satenv.h)
  * GAE scan, Gaussian sampling: HIP kernels (include/satrl_rollout.h)
  * Gaussian actor / critic / clipped-surrogate update: PyTorch-ROCm
  * data parallel: one process per GPU, RCCL over xGMI
"""
from ._lib import NativeError, build, lib  # noqa: F401

__all__ = ["NativeError", "build", "lib"]
