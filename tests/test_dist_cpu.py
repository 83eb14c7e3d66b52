"""Data-parallel path on CPU with gloo, world_size 2: bucketed gradient
all-reduce, the rank batch partition, and one multi-GPU-style epoch giving the
same parameters as averaging the two batches' gradients in one process."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch.utils.data import DataLoader, TensorDataset

WORLD = 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n=8, T=16):
    g = torch.Generator().manual_seed(5)
    return TensorDataset(torch.randn(n, T, 256, generator=g), torch.randn(n, T, 61, generator=g) * 20)


def _loader(ds):
    return DataLoader(ds, batch_size=2, shuffle=True, generator=torch.Generator().manual_seed(9))


def _worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from neurosync_trainer_lite_amd import parallel
    from neurosync_trainer_lite_amd.utils.training_utils import rank_batches, train_one_epoch_multi_gpu
    from tests.oracle_module import OracleLoss, OracleSeq2Seq
    r, w, _ = parallel.init_from_env(backend="gloo")
    assert (r, w) == (rank, WORLD)
    # 1. bucketed SUM all-reduce, ragged tail
    g = torch.arange(1000, dtype=torch.float32) * (rank + 1)
    red = parallel.GradAllReducer(g, bucket_bytes=256 * 4)
    red.ready(600)
    red.finish()
    torch.testing.assert_close(g, torch.arange(1000, dtype=torch.float32) * 3)
    # 2. partition: rank r takes batches s*W + r of one common order
    ds = _data()
    dl = _loader(ds)
    order = list(_loader(ds).batch_sampler)
    mine = [b for _, b in rank_batches(dl, rank, WORLD)]
    assert len(mine) == len(order) // WORLD
    for s, (src, _) in enumerate(mine):
        torch.testing.assert_close(src, ds.tensors[0][order[s * WORLD + rank]])
    # 3. one epoch, replicated Adam on averaged gradients
    model = OracleSeq2Seq()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-5)
    steps = train_one_epoch_multi_gpu(0, [model], _loader(ds), OracleLoss(), opt, [torch.device("cpu")], clip=2.0,
                                      batch_step=0, total_epochs=1)
    assert steps == len(order) // WORLD
    torch.save({k: v.detach() for k, v in model.state_dict().items()}, os.path.join(out_dir, "r%d.pt" % rank))
    dist.destroy_process_group()


def test_data_parallel_gloo(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)  # plots go under dataset/validation_plots here
    mp.spawn(_worker, args=(_port(), str(tmp_path)), nprocs=WORLD, join=True)
    a = torch.load(tmp_path / "r0.pt", weights_only=True)
    b = torch.load(tmp_path / "r1.pt", weights_only=True)
    for k in a:
        torch.testing.assert_close(a[k], b[k], rtol=0, atol=0)
    # single-process equivalent: mean of the two batches' gradients per step
    from tests.oracle_module import OracleLoss, OracleSeq2Seq
    ds = _data()
    order = list(_loader(ds).batch_sampler)
    model = OracleSeq2Seq()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-5)
    crit = OracleLoss()
    for s in range(len(order) // WORLD):
        grads = None
        for r in range(WORLD):
            idx = order[s * WORLD + r]
            opt.zero_grad()
            crit(model(ds.tensors[0][idx]), ds.tensors[1][idx]).backward()
            gs = [p.grad.clone() for p in model.parameters()]
            grads = gs if grads is None else [x + y for x, y in zip(grads, gs)]
        for p, gsum in zip(model.parameters(), grads):
            p.grad = gsum / WORLD
        torch.nn.utils.clip_grad_norm_(model.parameters(), 2.0)
        opt.step()
    for k, v in model.state_dict().items():
        torch.testing.assert_close(a[k], v, rtol=1e-5, atol=1e-6)
