"""Train ImprovedNN on the reference's 841 reachable-domain golden pairs
(build container, CPU; the output is data, not code on the GPU box).

Follows the reference's offline trainer
single_pluse_model/single_pulse_fully_connected_model.py:263-350 step for step:
  * inputs  all_input.csv   [a, e, i, f, fuel]  -> StandardScaler (fit on all 841 rows, :273-277)
  * targets output_data.csv [xc, yc, a, b, theta] x 2 ellipses -> StandardScaler
  * random_split 90 / 10 (:288-290), DataLoader batch 16, shuffle (:293-294)
  * ImprovedNN (model.py:7-24, dropout 0.2 active while training), MSELoss,
    Adam lr 1e-3, StepLR(step 10, gamma 0.1) per epoch, 500 epochs (:306-326)
  * held-out MSE on the standardised targets (:329-337)
The reference seeds nothing; this script seeds torch with --seed (default 0),
so the split and the weights are reproducible.  Parity of the training
itself is unpinned: the reference holds no trained weights (MLPNet.pth is
not in it), only this recipe and the data.

Writes ppo-rl-satellite_amd/satrl/data/improvednn_trained.npz: the weights
(fc1..fc4 weight / bias, f32), the scalers (sklearn mean_ / scale_), the
split's held-out rows (inputs and targets, the fixture the GPU test checks the
kernel against) and the losses.  satrl.surrogate.Surrogate.load_trained packs
it with the scalers in the blob (satenv_surrogate_set_scalers), so
satenv_surrogate emits real ellipse parameters.

    python tools/train_improvednn.py [--seed 0] [--epochs 500]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = "/root/reference/single_pluse_model"
OUT = os.path.join(ROOT, "ppo-rl-satellite_amd", "satrl", "data", "improvednn_trained.npz")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--epochs", type=int, default=500)
    ap.add_argument("--out", default=OUT)
    a = ap.parse_args()
    import pandas as pd
    import torch
    from sklearn.preprocessing import StandardScaler
    from torch.utils.data import DataLoader, TensorDataset, random_split
    sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))
    from satrl.surrogate import ImprovedNNDropout

    torch.manual_seed(a.seed)
    torch.set_num_threads(1)
    x_raw = pd.read_csv(os.path.join(REF_DIR, "all_input.csv")).values
    y_raw = pd.read_csv(os.path.join(REF_DIR, "output_data.csv")).values
    in_sc, out_sc = StandardScaler(), StandardScaler()
    x = torch.tensor(in_sc.fit_transform(x_raw), dtype=torch.float32)
    y = torch.tensor(out_sc.fit_transform(y_raw), dtype=torch.float32)
    ds = TensorDataset(x, y)
    n_train = int(0.9 * len(ds))
    train, test = random_split(ds, [n_train, len(ds) - n_train])
    train_loader = DataLoader(train, batch_size=16, shuffle=True)
    test_loader = DataLoader(test, batch_size=16, shuffle=False)
    net = ImprovedNNDropout()
    crit = torch.nn.MSELoss()
    opt = torch.optim.Adam(net.parameters(), lr=0.001)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=10, gamma=0.1)
    losses = []
    for ep in range(a.epochs):
        net.train()
        tot = 0.0
        for xb, yb in train_loader:
            opt.zero_grad()
            loss = crit(net(xb), yb)
            loss.backward()
            opt.step()
            tot += loss.item()
        sched.step()
        losses.append(tot / len(train_loader))
        if (ep + 1) % 10 == 0:
            print(f"Epoch {ep + 1}/{a.epochs}, Loss: {losses[-1]}")
    net.eval()
    test_loss = 0.0
    with torch.no_grad():
        for xb, yb in test_loader:
            test_loss += crit(net(xb), yb).item()
    test_loss /= len(test_loader)
    ti = np.asarray(test.indices, dtype=np.int64)
    with torch.no_grad():
        pred = out_sc.inverse_transform(net(x[ti]).numpy().astype(np.float64))
    true = y_raw[ti]
    rel = np.abs(pred - true) / np.maximum(np.abs(true), 1e-12)
    print(f"Test Loss: {test_loss}  (standardised MSE, {len(ti)} held-out rows)")
    print("held-out median relative error per output:", np.round(np.median(rel, axis=0), 4).tolist())
    sd = {k: v.detach().numpy().astype(np.float32) for k, v in net.state_dict().items()}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    np.savez(a.out, **{k.replace(".", "_"): v for k, v in sd.items()},
             in_mean=in_sc.mean_, in_scale=in_sc.scale_, out_mean=out_sc.mean_, out_scale=out_sc.scale_,
             test_idx=ti, test_x=x_raw[ti], test_y=true, train_losses=np.asarray(losses),
             test_loss=np.float64(test_loss), seed=np.int64(a.seed), epochs=np.int64(a.epochs))
    print("wrote", a.out)


if __name__ == "__main__":
    main()
