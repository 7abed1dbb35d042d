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
import ctypes as C
import os

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr

# ImprovedNN trained on the reference's 841 golden pairs by the reference's
# own recipe (tools/train_improvednn.py, single_pulse_fully_connected_model.py:
# 263-350): weights + StandardScalers + the held-out split
TRAINED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "improvednn_trained.npz")


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


def load_trained(path=TRAINED):
    """(state_dict, scalers) of a tools/train_improvednn.py bundle; scalers =
    (in_mean, in_scale, out_mean, out_scale) f64, sklearn's mean_ / scale_."""
    with np.load(path, allow_pickle=False) as z:
        sd = {f"fc{k}.{w}": torch.from_numpy(z[f"fc{k}_{w}"]) for k in range(1, 5) for w in ("weight", "bias")}
        sc = tuple(np.asarray(z[n], dtype=np.float64) for n in ("in_mean", "in_scale", "out_mean", "out_scale"))
    return sd, sc


class Surrogate:
    """Packed bf16 copy of an ImprovedNN on the device + the env-path kernel.
    state_dict: None (random init from `seed`), a state_dict or .pth path, or
    "trained" (the committed net trained on the reference's golden pairs,
    with its StandardScalers in the blob: outputs are ellipse parameters)."""

    def __init__(self, device="cuda", seed=0, state_dict=None):
        self.device = torch.device(device)
        g = torch.random.fork_rng(devices=[])
        with g:
            torch.manual_seed(seed)
            self.net = ImprovedNN()
        self.scalers = None
        if isinstance(state_dict, str) and state_dict == "trained":
            state_dict, self.scalers = load_trained()
        if state_dict is not None:
            self.load_state_dict(state_dict, scalers=self.scalers)
        self.net.to(self.device)
        self.blob = torch.empty(_lib.lib().satenv_surrogate_blob_bytes(), dtype=torch.uint8, device=self.device)
        self.pack()

    def load_state_dict(self, sd, scalers=None):
        """A state_dict or a path to one (loaded with weights_only=True).
        `scalers` (in_mean, in_scale, out_mean, out_scale) go with these
        weights; None loads them without scalers (identity), so weights
        loaded into a Surrogate built from the trained net do not keep that
        net's StandardScalers."""
        self.scalers = None if scalers is None else tuple(scalers)
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
        if self.scalers is not None:
            self.set_scalers(*self.scalers)

    def set_scalers(self, in_mean, in_scale, out_mean, out_scale):
        """The trainer's StandardScalers (sklearn mean_ / scale_) into the blob:
        features are standardised before the bf16 input layer and fc4's
        output is mapped back (satenv_surrogate_set_scalers)."""
        arrs = [np.ascontiguousarray(v, dtype=np.float64) for v in (in_mean, in_scale, out_mean, out_scale)]
        if [a.size for a in arrs] != [5, 5, 10, 10]:
            raise ValueError("scalers: in_mean/in_scale of 5, out_mean/out_scale of 10")
        self.scalers = tuple(arrs)
        check(_lib.lib().satenv_surrogate_set_scalers(ptr(self.blob), *[a.ctypes.data_as(C.c_void_p) for a in arrs],
                                                      stream_ptr()), "satenv_surrogate_set_scalers")

    def reference_forward(self, x):
        """fp32 torch forward of the same network incl. the scalers (f64
        standardisation as sklearn), the numerics reference of the kernel."""
        xs = x.double()
        if self.scalers is not None:
            im, isc, om, osc = (torch.as_tensor(v, device=x.device) for v in self.scalers)
            xs = (xs - im) / isc
        y = self.net(xs.float()).double()
        if self.scalers is not None:
            y = y * osc + om
        return y.float()

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


# ---------------------------------------------------------------------------
# Flag 2: the ellipse-fitting network trainer the env owns
# (environment.py:49, :298-301; real_time_data_process.py:127-183)
# ---------------------------------------------------------------------------
class ImprovedNNDropout(ImprovedNN):
    """ImprovedNN with model.py:14's Dropout(0.2) after fc1 and fc2, as the
    reference trains it (the module is in training mode)."""

    def __init__(self):
        super().__init__()
        self.dropout = torch.nn.Dropout(0.2)

    def forward(self, x):
        x = self.dropout(torch.relu(self.fc1(x)))
        x = self.dropout(torch.relu(self.fc2(x)))
        x = torch.relu(self.fc3(x))
        return self.fc4(x)


def rtp_orbital_elements(miu, R0, V0):
    """real_time_data_process.calculate_orbital_elements (:11-105) on host
    arrays: [a, e, i, omega, Omega, f] (ellipse/hyperbola), [a, i, u, Omega]
    (circular) or [p, i, omega, Omega, f] (parabolic), numpy semantics."""
    R0 = np.asarray(R0)
    V0 = np.asarray(V0)
    r_norm = np.linalg.norm(R0)
    v_norm = np.linalg.norm(V0)
    r_dot_v = np.dot(R0, V0)
    en = 2 / r_norm - v_norm ** 2 / miu
    a = 1 / abs(en) if en != 0 else None
    E = (v_norm ** 2 / miu - 1 / r_norm) * R0 - r_dot_v / miu * V0
    e = np.linalg.norm(E)
    H = np.cross(R0, V0)
    h = np.linalg.norm(H)
    p = h ** 2 / miu
    Z, X, Y = np.array([0, 0, 1]), np.array([1, 0, 0]), np.array([0, 1, 0])
    N = np.cross(Z, H)
    n = np.linalg.norm(N)
    with np.errstate(invalid="ignore", divide="ignore"):
        i = np.arccos(np.dot(Z, H) / h)
        if e != 0:
            omega = np.arccos(np.dot(N, E) / n / e) if (n != 0 and e != 0) else 0.0
            if np.dot(Z, E) < 0:
                omega = 2 * np.pi - omega
        else:
            u = np.arccos(np.dot(N, R0) / n / r_norm)
            if np.dot(R0, Z) < 0:
                u = 2 * np.pi - u
        Omega = np.arccos(np.dot(X, N) / n) if n != 0 else 0.0
        if np.dot(Y, N) < 0:
            Omega = 2 * np.pi - Omega
        if e != 0:
            f = np.arccos(np.dot(E, R0) / e / r_norm)
            if r_dot_v < 0:
                f = 2 * np.pi - f
    if en != 0:
        return [a, e, i, omega, Omega, f] if e != 0 else [a, i, u, Omega]
    return [p, i, omega, Omega, f]


class network_method_train:  # noqa: N801  (reference class name)
    """Drop-in for real_time_data_process.network_method_train (:127-183):
    one Adam step (lr 1e-3, StepLR 10 / 0.1) of ImprovedNN on the
    StandardScaler-transformed (input, target) of the current step.  A
    one-row StandardScaler maps every finite value to 0, so the reference
    trains the net towards f(0) = 0 whatever the ellipse is; the step runs
    on torch's CPU like the reference's, drawing ImprovedNN's init and the
    dropout masks from the same global generator in the same order.

    Divergence by necessity: every 10th step the reference saves MLPNet2.pth
    to the author's absolute path (/mnt/datab/...), which raises anywhere
    else; here it goes to `save_dir` (None: not saved)."""

    def __init__(self, pretrain=False, pretrained_path=None, save_dir=None):
        from sklearn.preprocessing import StandardScaler
        self.net = ImprovedNNDropout()
        if pretrain:
            if pretrained_path is None:
                raise FileNotFoundError("pretrain=True needs pretrained_path (MLPNet.pth; the reference's path is "
                                        "an absolute one on the author's machine)")
            sd = torch.load(pretrained_path, map_location="cpu", weights_only=True)
            self.net.load_state_dict(sd)
        self.criterion = torch.nn.MSELoss()
        self.optimizer = torch.optim.Adam(self.net.parameters(), lr=0.001)
        self.scheduler = torch.optim.lr_scheduler.StepLR(self.optimizer, step_size=10, gamma=0.1)
        self.count = 0
        self.loss = []
        self.all_loss = []
        self.save_dir = save_dir
        self.input_scaler = StandardScaler()
        self.output_scaler = StandardScaler()

    def train(self, R0, V0, fuel, target):
        target = self.output_scaler.fit_transform(np.asarray(target).reshape(1, -1))
        target = torch.tensor(target.reshape(10), dtype=torch.float32)
        orbit_data = rtp_orbital_elements(3.986e14, R0, V0)
        x = orbit_data[:3] + orbit_data[5:]
        x.append(fuel)
        x = self.input_scaler.fit_transform(np.array(x).reshape(1, -1)).reshape(5)
        x = torch.tensor(x, dtype=torch.float32)
        self.optimizer.zero_grad()
        predictions = self.net(x)
        loss = self.criterion(predictions, target)
        self.loss.append(loss)
        self.all_loss.append(loss)
        loss.backward()
        self.optimizer.step()
        self.count += 1
        if self.count == 10:
            self.scheduler.step()
            self.count = 0
            print("loss: ", sum(self.loss) / 10)
            self.loss = []
            if self.save_dir is not None:
                import os
                torch.save(self.net.state_dict(), os.path.join(self.save_dir, "MLPNet2.pth"))
