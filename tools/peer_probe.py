#!/usr/bin/env python3
"""Development probe (not shipped): the peer all-reduce's stages on a
1-GPU box, two ranks on cuda:0 over gloo, each stage logged with a
timestamp to gpurun_out/peer_probe_r<rank>.log (appended as it goes)."""
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-rl-satellite_amd"))


def rank_main(rank, port, world):
    log = open(os.path.join(ROOT, "gpurun_out", f"peer_probe_r{rank}.log"), "a", buffering=1)
    t0 = time.time()

    def say(m):
        log.write(f"{time.time() - t0:8.3f} r{rank} {m}\n")

    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    say("pg up")
    from satrl.peer import PeerComm
    from satrl.ppo import ppo_layout
    n = ppo_layout(int(os.environ.get("PROBE_H", "64")))["total"]
    H = int(os.environ.get("PROBE_H", "64"))
    pc = PeerComm(dist.group.WORLD, n, "cuda:0", H)
    say(f"peer comm up, n {n}, bufs {[hex(b or 0) for b in pc.bufs]}")
    G = torch.full((n,), float(rank + 1), device="cuda:0")
    nsq = torch.zeros(2 * 1024, dtype=torch.float64, device="cuda:0")
    steps = torch.zeros(2, dtype=torch.float64, device="cuda:0")
    for k in range(3):
        G.fill_(float(rank + 1))
        pc.all_reduce_dp_(H, 256, G, nsq, steps)
        say(f"call {k} queued")
        torch.cuda.synchronize()
        say(f"call {k} done: G[0] {G[0].item()} G[-1] {G[-1].item()} err {pc.error()} steps {steps.tolist()}")
    dist.barrier()
    pc.close()
    say("closed")
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(os.environ.get("PROBE_W", "2"))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(rank_main, args=(port, world), nprocs=world, start_method="spawn")
    print("peer probe done")
