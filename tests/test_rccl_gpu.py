"""The data-parallel collectives through RCCL on one MI355X.

One GPU cannot host two RCCL ranks, so the nccl (= RCCL) backend runs here as a
world_size-1 process group: every collective the multi-GPU step issues
(ShardComm.reduce_scatter / all_gather of the sharded optimizer, the bucketed
GradAllReducer of NSTL_DP=allreduce, the clip-norm all_reduce) executes through
RCCL on the device.  The same programme on a world_size-1 gloo group must give
bit-identical parameters, and both must match a plain single-process step
(reference step: utils/training_utils.py:56-80; multi-GPU replaced:
utils/training_utils.py:176-263).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
STEPS = 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(seed=5):
    from neurosync_trainer_lite_amd.config import training_config
    from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components
    cfg = dict(training_config)
    cfg.update(hidden_dim=256, num_heads=4, n_layers=1, dropout=0.0, use_amp=True)
    torch.manual_seed(seed)
    model = build_model(cfg, "cuda:0")
    crit, opt, _ = prepare_training_components(cfg, model)
    return model, crit, opt


def _batch(i):
    g = torch.Generator().manual_seed(300 + i)
    return torch.randn(4, 64, 256, generator=g).cuda(), (torch.randn(4, 64, 61, generator=g) * 20).cuda()


def _train(model, crit, opt):
    model.train()
    for s in range(STEPS):
        src, trg = _batch(s)
        opt.zero_grad()
        crit(model(src), trg).backward()
        opt.step(max_norm=2.0)
    torch.cuda.synchronize()


def _worker(rank, backend, port, out):
    from neurosync_trainer_lite_amd import parallel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=0, world_size=1)
    res = {"backend": dist.get_backend()}
    # 1. the sharded optimizer's collectives on a raw arena
    n = 64 * 840 * 3
    torch.manual_seed(11)
    full = torch.randn(n, device="cuda:0")
    comm = parallel.ShardComm(n)
    shard = torch.empty(comm.shard, device="cuda:0")
    comm.reduce_scatter(full, shard)
    gathered = full.clone()
    gathered[comm.lo:comm.hi] = shard * 2
    comm.all_gather(gathered)
    res["rs"], res["ag"] = shard.cpu(), gathered.cpu()
    # 2. bucketed all-reduce over a gradient arena (small buckets: several launches)
    torch.manual_seed(12)
    g = torch.randn(10000, device="cuda:0")
    red = parallel.GradAllReducer(g, bucket_bytes=4096, min_world=1)
    red.ready(5000)
    red.ready(7001)
    red.finish()
    res["ar"] = g.cpu()
    # 3. the sharded (ZeRO-1) training step through the engine
    model, crit, opt = _model()
    model(_batch(0)[0])  # build the engine
    opt.shard()
    _train(model, crit, opt)
    opt.consolidate()
    res["zero1"] = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    # 4. the bucketed all-reduce step (NSTL_DP=allreduce): reducer forced on one rank
    model, crit, opt = _model()
    model(_batch(0)[0])
    model.engine().grad_reducer = parallel.GradAllReducer(model.engine().g32, bucket_bytes=1 << 20, min_world=1)
    _train(model, crit, opt)
    res["allreduce"] = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    torch.save(res, out)
    dist.destroy_process_group()


def test_rccl_collectives_match_gloo_and_single_process(tmp_path):
    outs = {}
    for backend in ("nccl", "gloo"):
        outs[backend] = str(tmp_path / ("%s.pt" % backend))
        mp.spawn(_worker, args=(backend, _port(), outs[backend]), nprocs=1, join=True)
    r = torch.load(outs["nccl"], weights_only=True)
    q = torch.load(outs["gloo"], weights_only=True)
    assert r["backend"] == "nccl" and q["backend"] == "gloo"
    for key in ("rs", "ag", "ar"):
        assert torch.equal(r[key], q[key]), key
    for mode in ("zero1", "allreduce"):
        for k in r[mode]:
            assert torch.equal(r[mode][k], q[mode][k]), (mode, k)
    # world 1: reduce-scatter is the identity, all-gather returns the shard in place
    n = r["ag"].numel()
    assert torch.equal(r["ag"], r["rs"] * 2) and r["rs"].numel() == n
    # and the distributed programmes equal a plain single-process step
    model, crit, opt = _model()
    _train(model, crit, opt)
    plain = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    for mode in ("zero1", "allreduce"):
        for k, v in plain.items():
            torch.testing.assert_close(r[mode][k], v, rtol=1e-6, atol=1e-7, msg=lambda m: "%s %s: %s" % (mode, k, m))
