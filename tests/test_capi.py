"""CPU checks of the C-ABI boundary: the library loads and exports every
symbol the public headers declare (no compute calls: no GPU here)."""
import ctypes as C
import os
import re

import pytest

from conftest import ROOT


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    return set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(sat\w+)\s*\(", txt, re.M))


def test_headers_declare_expected_entry_points():
    env = _declared("satenv.h")
    assert {"satenv_create", "satenv_reset", "satenv_step", "satenv_step_autoreset", "satenv_destroy",
            "satenv_get_state", "satenv_set_state", "satenv_last_error"} <= env
    assert {"satrl_gae", "satrl_gaussian_sample", "satrl_moments"} <= _declared("satrl_rollout.h")
    assert {"satrl_ppo_rowpass", "satrl_ppo_reduce", "satrl_ppo_adam", "satrl_ppo_layout"} <= _declared("satrl_ppo.h")
    assert {"satrl_peer_alloc", "satrl_peer_open", "satrl_ppo_allreduce_peer"} <= _declared("satrl_peer.h")
    # the host build exports every env entry point of satenv.h it restates, same signature, satenv_cpu_ prefix
    cpu = _declared("satenv_cpu.h")
    assert {n.replace("satenv_", "satenv_cpu_", 1) for n in ("satenv_create", "satenv_destroy", "satenv_num_envs",
            "satenv_set_params", "satenv_reset", "satenv_step", "satenv_step_autoreset", "satenv_get_state",
            "satenv_set_state", "satenv_danger_zone", "satenv_check", "satenv_last_error")} == cpu


def test_library_exports_every_declared_symbol():
    import satrl._lib as L
    if not os.path.exists(L.LIB_PATH):
        L.build()
    lib = L.lib()          # loads with torch's HIP runtime; no device needed
    declared = (_declared("satenv.h") | _declared("satenv_cpu.h") | _declared("satrl_rollout.h") |
                _declared("satrl_ppo.h") | _declared("satrl_peer.h"))
    for name in sorted(declared):
        assert hasattr(lib, name), name
    assert set(L.exported_symbols()) == declared


def test_host_helpers_without_gpu():
    import numpy as np
    import satrl._lib as L
    from satrl import env as E
    assert L.lib().satenv_abi_version() == 2
    p = E.default_params()
    assert p.max_episode_steps == 1000 and p.fuel_c0 == 320 and p.d_range == 100000
    # host STM equals the oracle's / reference's matrix bit for bit
    import oracle as O
    assert np.array_equal(E.stm(100.0), O.stm(100.0))


def test_entry_points_reject_bad_arguments_before_any_device_call():
    """Error behaviour of the boundary (include/*.h: 0 ok, negative codes):
    shapes, widths and null pointers are checked on the host before any HIP
    call, so these run without a GPU.  A non-null dummy pointer is never
    dereferenced on these paths."""
    import ctypes as C
    import satrl._lib as L
    from satrl import env as E
    lib = L.lib()
    fake = C.c_void_p(16)                       # never touched: every call below fails its host checks
    # satenv_create: null out / null params / num_envs <= 0 / bad propagator -> SATENV_ERR_ARG (-1)
    p = E.default_params()
    h = C.c_void_p()
    assert lib.satenv_create(None, 4, C.byref(p), 0) == -1
    assert lib.satenv_create(C.byref(h), 4, None, 0) == -1
    assert lib.satenv_create(C.byref(h), 0, C.byref(p), 0) == -1
    assert b"bad arguments" in lib.satenv_last_error()
    bad = E.default_params()
    bad.propagator = 7
    assert lib.satenv_create(C.byref(h), 4, C.byref(bad), 0) == -1
    assert b"propagator" in lib.satenv_last_error()
    assert lib.satenv_set_step_kernel(None, 2, 64) == -1 and lib.satenv_set_step_kernel(fake, 3, 64) == -1
    assert lib.satenv_set_step_kernel(fake, 2, 48) == -1                       # 16 / 32 / 64 envs per workgroup
    # learner side: unsupported hidden width, empty minibatch, net out of range, null buffers
    off = (C.c_int64 * 16)()
    assert lib.satrl_ppo_layout(100, off) == -1 and lib.satrl_ppo_layout(256, off) == 0
    assert lib.satrl_ppo_sizes(256, 0, None, None) == -1
    args = [fake, None, fake, fake, 0.1, 0.01, 1.6, fake, fake, fake, fake, None]
    assert lib.satrl_ppo_rowpass(100, 64, -1, *args) == -1                     # H not 64/128/256
    assert lib.satrl_ppo_rowpass(256, 0, -1, *args) == -1                      # empty minibatch
    assert lib.satrl_ppo_rowpass(256, 64, 2, *args) == -1                      # net not -1/0/1
    assert lib.satrl_ppo_rowpass(256, 64, -1, None, *args[1:]) == -1           # null rows
    big = 1 << 40                                # a p2 / plane capacity no call exceeds
    assert lib.satrl_ppo_dw2(256, 4096, -1, 0, fake, fake, fake, big, None) == -1   # S < 1
    assert lib.satrl_ppo_dw2(256, 64, -1, 64, fake, fake, fake, big, None) == -1    # an empty split
    assert lib.satrl_ppo_reduce(256, 64, -1, 1, 4, fake, big, fake, fake, fake, fake, fake, None) == -1   # mode
    assert lib.satrl_ppo_reduce(256, 64, -1, 1, 2, fake, big, fake, fake, fake, None, None, None) == -1   # no nsq
    assert lib.satrl_gae(0, 4, fake, fake, fake, 0.99, 0.95, fake, fake, None) == -1
    assert lib.satrl_gae(4, 4, fake, None, fake, 0.99, 0.95, fake, fake, None) == -1
    assert lib.satrl_policy_act(256, 8, fake, fake, fake, 1.6, 0, 0, 0, None, fake, fake, None, None,
                                None) == -1                                   # second agent without outputs
    assert lib.satrl_ppo_tanh(0, fake, fake, None) == -1
    # the fc2 operand image and the k-packed dW2 path (H = 256, mb above the 16-row threshold)
    assert lib.satrl_ppo_w2x_floats(256) == 2 * 256 * 256                    # the f32 W2^T at every width
    assert lib.satrl_ppo_w2x_floats(64) == 2 * 64 * 64
    assert lib.satrl_ppo_w2x_floats(100) == -1
    assert lib.satrl_ppo_w2x_sync(100, -1, fake, fake, None) == -1 and lib.satrl_ppo_w2x_sync(256, -1, None, fake, None) == -1
    assert lib.satrl_ppo_kx_elems(256, 4096) == 2 * 3 * 4096 * 256 and lib.satrl_ppo_kx_elems(256, 1500) == 6 * 1504 * 256
    assert lib.satrl_ppo_kx_elems(64, 4096) == -1
    kx_args = args[:9] + [big] + args[9:]        # (H1x, dZ2x, kx_elems, ptail, pw1, stream)
    assert lib.satrl_ppo_rowpass_kx(256, 512, -1, None, *kx_args[1:]) == -1     # null rows (16-row kernel's minibatch)
    assert lib.satrl_ppo_rowpass_kx(64, 4096, -1, *kx_args) == -1               # H 256 only
    assert lib.satrl_ppo_dw2_kx_splits(256, 4096, -1) == 8 and lib.satrl_ppo_dw2_kx_splits(256, 4096, 0) == 16
    assert lib.satrl_ppo_dw2_kx(256, 4096, -1, 0, fake, fake, big, fake, big, None) == -1     # S < 1
    assert lib.satrl_ppo_dw2_kx(256, 64, -1, 3, fake, fake, big, fake, big, None) == -1       # an empty split (2 chunks)
    assert lib.satrl_ppo_dw2_kx(256, 4096, -1, 8, None, fake, big, fake, big, None) == -1     # null H1x
    w1a = [fake, fake, big, fake, big]                     # (H1x, dZ2x, kx_elems, p2, p2_floats)
    assert lib.satrl_ppo_dw2_kx_w1(256, 4096, -1, 8, *w1a, 2, fake, fake, fake, fake, None) == -1   # mode 1 or 3
    assert lib.satrl_ppo_dw2_kx_w1(256, 4096, -1, 8, *w1a, 3, None, fake, fake, fake, None) == -1   # null p1
    assert lib.satrl_ppo_dw2_kx_w1(256, 4096, -1, 8, *w1a, 3, fake, fake, fake, None, None) == -1   # mode 3: nsq
    assert lib.satrl_ppo_dw2_kx_w1(64, 4096, -1, 8, *w1a, 1, fake, fake, fake, None, None) == -1    # H 256 only
    assert lib.satrl_ppo_reduce(256, 4096, -1, 8, 6, fake, big, None, None, fake, fake, fake, None) == -1  # 4 needs 1
    assert lib.satrl_ppo_rowpass_error(None, 1.0, None) == -1                 # the column-split kernel's error word
    assert lib.satrl_ppo_rowpass_error(C.byref(C.c_int()), 0.0, None) == -1  # no deadline
    assert lib.satrl_ppo_rowpass_fault_inject(-1, 0, None) == -1 and lib.satrl_ppo_rowpass_fault_inject(1 << 20, 0, None) == -1
    # the peer all-reduce: grid, deadline, buffers
    bufs = (C.c_void_p * 2)(16, 16)
    pa = [C.cast(bufs, C.c_void_p), fake, fake, fake]
    assert lib.satrl_ppo_allreduce_peer(256, 512, 2, 0, *pa, 0, 10.0, None) == -1            # no blocks
    assert lib.satrl_ppo_allreduce_peer(256, 512, 2, 0, *pa, 2048, 10.0, None) == -1         # > kPeerMaxBlocks
    assert lib.satrl_ppo_allreduce_peer(256, 512, 2, 0, *pa, 256, 0.0, None) == -1           # no deadline
    assert lib.satrl_ppo_allreduce_peer(256, 512, 2, 2, *pa, 256, 10.0, None) == -1          # rank >= world
    assert lib.satrl_ppo_allreduce_peer(256, 512, 9, 0, *pa, 256, 10.0, None) == -1          # world > 8
    assert lib.satrl_peer_blocks(100, C.byref(C.c_int())) == -1 and lib.satrl_peer_blocks(256, None) == -1
    assert lib.satrl_peer_error(None, C.byref(C.c_uint64()), None) == -1
    assert lib.satrl_peer_reset(fake, 8, None) == -1                                         # smaller than the header


def test_capi_refuses_calls_past_the_callers_buffers():
    """Round-5 fault (a dW2 run with more splits than its slabs were sized
    for wrote past p2): every call that writes or reads the dW2 slabs or the
    k-packed planes takes the caller's capacity and refuses with -1 before
    any launch (fake pointers, never touched; a launch would fail with -2 on
    this GPU-less host instead)."""
    import ctypes as C
    import satrl._lib as L
    lib = L.lib()
    fake = C.c_void_p(16)
    H, mb = 256, 4096
    S = lib.satrl_ppo_dw2_kx_splits(H, mb, -1)                    # 8
    kx = lib.satrl_ppo_kx_elems(H, mb)
    p2_8 = 2 * 8 * H * H                                         # slabs sized for 8 splits
    # an oversize split count (the round-5 case: 16 splits into slabs for 8)
    assert lib.satrl_ppo_dw2_kx(H, mb, -1, 16, fake, fake, kx, fake, p2_8, None) == -1
    assert b"p2 holds" in lib.satrl_ppo_last_error()
    assert lib.satrl_ppo_reduce(H, mb, -1, 16, 3, fake, p2_8, fake, fake, fake, fake, fake, None) == -1
    assert b"p2 holds" in lib.satrl_ppo_last_error()
    assert lib.satrl_ppo_dw2(H, mb, -1, 16, fake, fake, fake, p2_8, None) == -1
    # one net: the actor passes half, the critic (second half) the whole buffer
    assert lib.satrl_ppo_dw2_kx(H, mb, 1, S, fake, fake, kx, fake, p2_8 // 2, None) == -1
    # undersized planes, for the rowpass that writes them and the dW2 that reads them
    assert lib.satrl_ppo_rowpass_kx(H, mb, -1, fake, None, fake, fake, 0.1, 0.01, 1.6, fake, fake, kx - 1, fake,
                                    fake, None) == -1
    assert b"planes hold" in lib.satrl_ppo_last_error()
    assert lib.satrl_ppo_dw2_kx(H, mb, -1, S, fake, fake, kx - 1, fake, p2_8, None) == -1
    # H 64: one slab per 32-row block (128 at mb 4096) written by the fused rowpass
    assert lib.satrl_ppo_rowpass_dw2(64, mb, -1, fake, None, fake, fake, 0.1, 0.01, 1.6, fake, 2 * 127 * 64 * 64,
                                     fake, fake, None) == -1
    assert b"p2 holds" in lib.satrl_ppo_last_error()


def test_product_has_no_cpu_fallback():
    import torch
    from satrl import env as E
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(Exception):
        E.VecSatellites(4)


def test_reference_module_name_shims():
    """`from environment import satellites` etc. (CPPO_main.py:5-7) resolve to the engine."""
    import importlib
    import sys
    from conftest import PKG_DIR
    sys.path.insert(0, str(PKG_DIR))
    try:
        env = importlib.import_module("environment")
        ppo = importlib.import_module("ppo_continuous")
        rb = importlib.import_module("replaybuffer")
        main = importlib.import_module("CPPO_main")
    finally:
        sys.path.remove(str(PKG_DIR))
    import satrl.buffer
    import satrl.env
    import satrl.ppo
    import satrl.trainer
    assert env.satellites is satrl.env.satellites
    assert ppo.PPO_continuous is satrl.ppo.PPO_continuous
    assert rb.ReplayBuffer is satrl.buffer.ReplayBuffer
    assert main.args_param is satrl.trainer.args_param
    assert main.train_pursuer_network is satrl.trainer.train_pursuer_network


def test_improvednn_matches_reference_state_dict():
    """satrl.surrogate.ImprovedNN has the reference's parameter names/shapes:
    MLPNet2.pth (single_pluse_model/) loads with weights_only=True.  Runs only
    where the reference checkout exists (the build container)."""
    import os
    import torch
    path = "/root/reference/single_pluse_model/MLPNet2.pth"
    if not os.path.exists(path):
        pytest.skip("reference checkout not present")
    from satrl.surrogate import ImprovedNN
    sd = torch.load(path, map_location="cpu", weights_only=True)
    net = ImprovedNN()
    net.load_state_dict(sd)
    out = net(torch.zeros(1, 5))
    assert out.shape == (1, 10) and torch.isfinite(out).all()


def test_w2x_image_host_statement():
    """The fc2 operand image's host statement (satrl.ppo.w2x_image, what
    satrl_ppo_w2x_sync writes): the f32 fc2.weight^T of both nets at every
    width, and w2x_decode recovers it bit for bit."""
    import torch
    from satrl.ppo import w2x_decode, w2x_image
    g = torch.Generator().manual_seed(0)
    for H in (64, 256):
        W2 = torch.randn(2 * H * H, generator=g) * torch.exp(torch.randn(2 * H * H, generator=g) * 4)
        img = w2x_image(W2, H)
        assert img.dtype == torch.float32 and img.numel() == 2 * H * H
        assert torch.equal(w2x_decode(img, H), W2.view(2, H, H).transpose(1, 2))


def test_uses_column_split():
    """Which updates need the exchange check (ppo_kernels.hip cs_fits: H 256,
    a minibatch or ragged tail of at most 1024 rows)."""
    from satrl.ppo import uses_column_split
    assert uses_column_split(256, 512, 8192) and uses_column_split(256, 1024, 8192)
    assert not uses_column_split(256, 4096, 8192)            # configs[1]-sized minibatches, no tail
    assert uses_column_split(256, 4096, 8192 + 100)           # a 100-row tail
    assert not uses_column_split(256, 4096, 8192 + 2000)      # a tail over 1024 rows
    assert uses_column_split(256, 4096, 700)                  # one minibatch of the whole 700 rows
    assert not uses_column_split(64, 512, 8192) and not uses_column_split(128, 512, 8192)
