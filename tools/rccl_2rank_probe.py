"""Can two RCCL ranks share one MI355X?  Two processes on cuda:0 join a
world_size-2 nccl (= RCCL) group and run an all_reduce, a reduce_scatter_tensor
and an all_gather_into_tensor of 64 MB; each prints what it got.  If RCCL
refuses a second rank on one device the error is printed and the probe exits
non-zero.  python tools/rccl_2rank_probe.py"""
import os
import socket
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    try:
        dist.init_process_group("nccl", rank=rank, world_size=2, device_id=torch.device("cuda", 0))
        n = 16 << 20
        x = torch.full((n,), float(rank + 1), device="cuda:0")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        ok_ar = bool((x == 3.0).all().item())
        y = torch.arange(n, device="cuda:0", dtype=torch.float32) * (rank + 1)
        out = torch.empty(n // 2, device="cuda:0")
        dist.reduce_scatter_tensor(out, y)
        ref = torch.arange(n, device="cuda:0", dtype=torch.float32)[rank * (n // 2):(rank + 1) * (n // 2)] * 3
        ok_rs = bool(torch.equal(out, ref))
        g = torch.empty(n, device="cuda:0")
        dist.all_gather_into_tensor(g, out)
        ok_ag = bool(torch.equal(g, torch.arange(n, device="cuda:0", dtype=torch.float32) * 3))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            dist.all_reduce(x)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 10 * 1e3
        print("rank %d: all_reduce %s reduce_scatter %s all_gather %s; 64 MB all_reduce %.3f ms"
              % (rank, ok_ar, ok_rs, ok_ag, ms), flush=True)
        dist.destroy_process_group()
    except Exception as e:  # report, do not hang the partner forever
        print("rank %d: %s: %s" % (rank, type(e).__name__, e), flush=True)
        sys.exit(3)


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, port)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    codes = [p.exitcode for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    print("exit codes", codes)
    sys.exit(0 if codes == [0, 0] else 1)
