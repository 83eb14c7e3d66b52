"""Sharded optimizer (ZeRO-1, FusedAdam.shard) through the real HIP kernels:
two ranks on cuda:0 (gloo carries the collectives: one GPU cannot host two RCCL
ranks) against one process stepping the mean gradient of the same two batches."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
WORLD = 2
STEPS = 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(seed=3):
    from neurosync_trainer_lite_amd.config import training_config
    from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components
    cfg = dict(training_config)
    cfg.update(hidden_dim=256, num_heads=4, n_layers=1, dropout=0.0, use_amp=True)
    torch.manual_seed(seed)
    model = build_model(cfg, "cuda:0")
    crit, opt, _ = prepare_training_components(cfg, model)
    return model, crit, opt


def _batch(i):
    g = torch.Generator().manual_seed(100 + i)
    return (torch.randn(2, 64, 256, generator=g).cuda(), (torch.randn(2, 64, 61, generator=g) * 20).cuda())


def _worker(rank, port, out_dir, mode="zero1"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK="0", NSTL_DP=mode)
    from neurosync_trainer_lite_amd import parallel
    from neurosync_trainer_lite_amd.utils.training_utils import attach_data_parallel
    parallel.init_from_env(backend="gloo")
    model, crit, opt = _setup()
    model.train()
    model(_batch(0)[0])  # build the engine
    attach_data_parallel(model, opt, WORLD)
    assert opt._comm is not None
    if mode == "zero1_push":
        assert isinstance(model.engine().grad_reducer, parallel.ShardPusher)
    for s in range(STEPS):
        src, trg = _batch(2 * s + rank)
        opt.zero_grad()
        crit(model(src), trg).backward()
        opt.step(max_norm=2.0)
    if mode == "zero1_push":
        # the first step's pushed sums were checked against the reduce-scatter
        # (ShardPusher.verify) and the exchange stayed on the copy engines
        assert opt.dp_check is not None and opt.dp_check["ok"], opt.dp_check
        assert isinstance(model.engine().grad_reducer, parallel.ShardPusher) and opt.dp_fallback is None
    with pytest.raises(RuntimeError, match="consolidate"):
        model.state_dict()
    opt.consolidate()
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    osd = opt.state_dict()
    torch.save({"params": sd, "m": osd["state"][3]["exp_avg"].cpu(), "norm": float(opt.last_norm.item())},
               os.path.join(out_dir, "%s%d.pt" % ("z" if mode == "zero1" else mode, rank)))
    red = model.engine().grad_reducer
    if hasattr(red, "close"):
        red.close()
    dist.destroy_process_group()


def test_sharded_optimizer_matches_single_process(tmp_path):
    mp.spawn(_worker, args=(_port(), str(tmp_path)), nprocs=WORLD, join=True)
    z0 = torch.load(tmp_path / "z0.pt", weights_only=True)
    z1 = torch.load(tmp_path / "z1.pt", weights_only=True)
    for k in z0["params"]:
        torch.testing.assert_close(z0["params"][k], z1["params"][k], rtol=0, atol=0)
    # one process: both batches' gradients accumulated at 1/2 each, one step
    model, crit, opt = _setup()
    model.train()
    model(_batch(0)[0])
    eng = model.engine()
    eng.grad_scale_t = torch.full((1,), 0.5, device="cuda:0")
    for s in range(STEPS):
        opt.zero_grad()
        for r in range(WORLD):
            src, trg = _batch(2 * s + r)
            crit(model(src), trg).backward()
        opt.step(max_norm=2.0)
    torch.cuda.synchronize()
    ref = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    for k, v in ref.items():
        torch.testing.assert_close(z0["params"][k], v, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(z0["m"], opt.state_dict()["state"][3]["exp_avg"].cpu(), rtol=1e-5, atol=1e-8)
    assert abs(z0["norm"] - float(opt.last_norm.item())) < 1e-4 * float(opt.last_norm.item())


def test_pushed_shards_bit_identical_to_zero1(tmp_path):
    """NSTL_DP=zero1_push through the real kernels and copy engines: two ranks on
    cuda:0 map each other's receive buffers by IPC handle, push their gradient
    slices with device-to-device copies on the copy engines
    (hipMemcpyDeviceToDeviceNoCU) during backward, and each owner sums its shard
    with nstl_shard_sum (own + the other rank's slot, and the clip norm's
    partials in the same pass).  At two ranks that is the reduce-scatter's one
    addition, so parameters, moments and the clip norm equal zero1's bit for
    bit."""
    for mode in ("zero1", "zero1_push"):
        mp.spawn(_worker, args=(_port(), str(tmp_path), mode), nprocs=WORLD, join=True)
    for r in range(WORLD):
        a = torch.load(tmp_path / ("z%d.pt" % r), weights_only=True)
        b = torch.load(tmp_path / ("zero1_push%d.pt" % r), weights_only=True)
        for k in a["params"]:
            assert torch.equal(a["params"][k], b["params"][k]), (r, k)
        assert torch.equal(a["m"], b["m"]), r
        assert a["norm"] == b["norm"], (a["norm"], b["norm"])
