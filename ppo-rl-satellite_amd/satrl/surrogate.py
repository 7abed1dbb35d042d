"""Config 5: the ImprovedNN reachable-domain surrogate in the env path (bf16).

single_pluse_model/model.py:7-24 defines ImprovedNN (5 -> 256 -> 128 -> 64 ->
10, ReLU, dropout 0.2); real_time_data_process.network_method_process
(:112-125) evaluates it on [a, e, i, f, fuel_c] of the pursuer's absolute
orbit; environment.py:158 would store the result as the env's
ellipse_params (commented out in the reference; no reward term uses it).

Here the network runs as one HIP kernel per env step (satenv_surrogate):
orbital elements in FP64 per env, then three bf16 MFMA layers with f32
accumulation whose activations never leave registers (surrogate_device.h).
Inference semantics: no dropout (the reference constructs the net fresh in
training mode, so its dropout would make the output random).
"""
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr


class ImprovedNN(torch.nn.Module):
    """Parameter names and shapes of single_pluse_model/model.py:7-24, so the
    reference's state_dict files (e.g. MLPNet2.pth) load unchanged."""

    def __init__(self):
        super().__init__()
        self.fc1 = torch.nn.Linear(5, 256)
        self.fc2 = torch.nn.Linear(256, 128)
        self.fc3 = torch.nn.Linear(128, 64)
        self.fc4 = torch.nn.Linear(64, 10)

    def forward(self, x):     # fp32 torch forward (eval semantics), used as the numerics reference
        x = torch.relu(self.fc1(x))
        x = torch.relu(self.fc2(x))
        x = torch.relu(self.fc3(x))
        return self.fc4(x)


class Surrogate:
    """Packed bf16 copy of an ImprovedNN on the device + the env-path kernel."""

    def __init__(self, device="cuda", seed=0, state_dict=None):
        self.device = torch.device(device)
        g = torch.random.fork_rng(devices=[])
        with g:
            torch.manual_seed(seed)
            self.net = ImprovedNN()
        if state_dict is not None:
            self.load_state_dict(state_dict)
        self.net.to(self.device)
        self.blob = torch.empty(_lib.lib().satenv_surrogate_blob_bytes(), dtype=torch.uint8, device=self.device)
        self.pack()

    def load_state_dict(self, sd):
        """A state_dict or a path to one (loaded with weights_only=True)."""
        if isinstance(sd, str):
            sd = torch.load(sd, map_location="cpu", weights_only=True)
        self.net.load_state_dict({k: v for k, v in sd.items() if not k.startswith("dropout")})
        if hasattr(self, "blob"):
            self.net.to(self.device)
            self.pack()

    def pack(self):
        ps = [t.detach().float().contiguous() for m in (self.net.fc1, self.net.fc2, self.net.fc3, self.net.fc4)
              for t in (m.weight, m.bias)]
        self._packed_from = ps          # keep alive until the pack kernel ran
        check(_lib.lib().satenv_surrogate_pack(*[ptr(t) for t in ps], ptr(self.blob), stream_ptr()),
              "satenv_surrogate_pack")

    def env_forward(self, env, out=None):
        """ellipse_params [N][10] f32 from the env's current pursuer state."""
        if out is None:
            out = torch.empty((env.num_envs, 10), dtype=torch.float32, device=self.device)
        _lib.require_cuda(out, torch.float32, (env.num_envs, 10), "out")
        check(_lib.lib().satenv_surrogate(env._h, ptr(self.blob), ptr(out), stream_ptr()), "satenv_surrogate")
        return out

    def forward(self, x, out=None):
        """The bf16 network on features x [n][5] f32."""
        n = x.shape[0]
        _lib.require_cuda(x, torch.float32, (n, 5), "x")
        if out is None:
            out = torch.empty((n, 10), dtype=torch.float32, device=self.device)
        check(_lib.lib().satenv_surrogate_mlp(n, ptr(x), ptr(self.blob), ptr(out), stream_ptr()), "satenv_surrogate_mlp")
        return out


def bf16_reference(net, x):
    """fp32 torch emulation of the kernel's rounding points: bf16 weights,
    inputs and post-ReLU activations, f32 accumulation and bias."""
    q = lambda t: t.to(torch.bfloat16).float()
    h = q(x)
    for i, m in enumerate((net.fc1, net.fc2, net.fc3, net.fc4)):
        h = h @ q(m.weight).t() + m.bias.float()
        if i < 3:
            h = q(torch.relu(h))
    return h
