"""Probe: can two RCCL ranks share ONE GPU on this box (both on cuda:0)? If RCCL accepts it, the RCCL code paths
(all_reduce, all_gather, all_to_all_single) can be exercised on a one-GPU box by multi-rank tests.

python tools/microbench/rccl_one_gpu_probe.py
"""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        x = torch.full((1024,), float(rank + 1), device="cuda")
        dist.all_reduce(x)
        g = [torch.empty(4, device="cuda") for _ in range(world)]
        dist.all_gather(g, torch.full((4,), float(rank), device="cuda"))
        a = torch.arange(world * 2, dtype=torch.float32, device="cuda") + 100 * rank
        b = torch.empty_like(a)
        dist.all_to_all_single(b, a)
        torch.cuda.synchronize()
        q.put((rank, "ok", float(x[0]), [float(t[0]) for t in g], b.tolist()))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, "error", repr(e)[:500]))


if __name__ == "__main__":
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 2
    ps = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    alive = [p.is_alive() for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    res = []
    while not q.empty():
        res.append(q.get())
    print("results:", res, "alive:", alive, flush=True)
    sys.exit(0)
