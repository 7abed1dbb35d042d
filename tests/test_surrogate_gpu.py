"""Config 5 on the MI355X: the ImprovedNN surrogate (single_pluse_model/
model.py:7-24) in bf16 through satenv_surrogate / satenv_surrogate_mlp.

Numerics bar: against a torch fp32 emulation of the kernel's rounding points
(bf16 weights, inputs and post-ReLU activations; f32 accumulation and bias,
satrl.surrogate.bf16_reference) the outputs agree to 1e-2 of the row's
largest magnitude (a different f32 summation order can flip a bf16 rounding
of a hidden activation); against the plain fp32 network to 5e-2 (bf16
quantisation of the inputs: a ~ 4e7 m keeps 8 mantissa bits).  Features
from the env state use the oracle's orbital elements (FP64, <= 1e-12).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def S():
    from satrl import surrogate
    return surrogate


def _feats(rng, n):
    return np.stack([rng.uniform(7e6, 5e7, n), rng.uniform(0.0, 0.8, n), rng.uniform(0.0, np.pi, n),
                     rng.uniform(0.0, 2 * np.pi, n), rng.uniform(0.0, 320.0, n)], 1).astype(np.float32)


def _close(got, ref, rtol):
    scale = ref.abs().amax(1, keepdim=True).clamp_min(1e-30)
    err = ((got - ref).abs() / scale).max().item()
    assert err < rtol, err
    return err


@pytest.mark.parametrize("n", [1, 16, 1000, 16384])
def test_mlp_bf16_vs_torch(S, n):
    sur = S.Surrogate(device="cuda:0", seed=1)
    x = torch.tensor(_feats(np.random.default_rng(n), n), device="cuda:0")
    got = sur.forward(x)
    _close(got, S.bf16_reference(sur.net, x), 1e-2)
    with torch.no_grad():
        _close(got, sur.net(x), 5e-2)


def test_mlp_small_inputs_and_layer_permutation(S):
    """Unit-scale inputs (the StandardScaler regime the reference trains in):
    every hidden neuron matters, so a wrong k permutation in the packed
    weights shows up at once."""
    sur = S.Surrogate(device="cuda:0", seed=2)
    x = torch.randn((512, 5), device="cuda:0")
    _close(sur.forward(x), S.bf16_reference(sur.net, x), 1e-2)


def test_env_path_features_and_forward(S, oracle):
    from satrl.env import VecSatellites
    n = 4096
    env = VecSatellites(n, device="cuda:0", d_capture=15000.0, max_episode_steps=1000)
    env.reset(0)
    g = torch.Generator(device="cuda:0").manual_seed(0)
    for _ in range(5):
        pa = torch.rand((n, 3), device="cuda:0", generator=g) * 3.2 - 1.6
        ea = torch.rand((n, 3), device="cuda:0", generator=g) * 3.2 - 1.6
        env.step_autoreset(pa, ea)
    sur = S.Surrogate(device="cuda:0", seed=3)
    out = sur.env_forward(env)
    f, _ = env.get_state()
    f = f.cpu().numpy()
    R_cw = np.array([27098000.0, 32306000.0, 0.0])
    V_cw = np.array([-2350.0, 1970.0, 0.0])
    feats = np.zeros((n, 5), dtype=np.float32)
    for k in range(n):
        rc, el = oracle.orbital_elements(R_cw + f[0:3, k], V_cw + f[3:6, k])
        assert rc == 0
        feats[k] = [el[0], el[1], el[2], el[5], f[12, k]]
    ref = S.bf16_reference(sur.net, torch.tensor(feats, device="cuda:0"))
    _close(out, ref, 1e-2)
