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


def _shard_worker(rank, port, out_dir, world=WORLD, overlap=False, push=False, accumulate=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from neurosync_trainer_lite_amd import parallel
    parallel.init_from_env(backend="gloo")
    ns = 64 * 840  # one ARENA_ALIGN unit: splits for 1..8 ranks
    n = ns + 192   # + a replicated tail (the arena's f32 vectors)
    comm = parallel.ShardComm(ns)
    assert (comm.shard, comm.lo) == (ns // world, rank * ns // world)
    g = torch.Generator().manual_seed(1)
    p = torch.randn(n, generator=g)
    m, v = torch.zeros(n), torch.zeros(n)
    grads = torch.randn(n, generator=torch.Generator().manual_seed(10 + rank)) * (rank + 1)
    gs = torch.empty(comm.shard)
    partial = torch.zeros(4)

    def sumsq_fn(x, part):
        part.zero_()
        part[0] = (x.double() ** 2).sum().float()

    def adam_fn(lo, k, x, part):
        coef = min(1.0, 2.0 / (float(part.sum()) ** 0.5 + 1e-6))
        gg = x * coef + 1e-5 * p[lo:lo + k]
        m[lo:lo + k] = 0.9 * m[lo:lo + k] + 0.1 * gg
        v[lo:lo + k] = 0.999 * v[lo:lo + k] + 0.001 * gg * gg
        p[lo:lo + k] -= 1e-3 / 0.1 * m[lo:lo + k] / ((v[lo:lo + k] / 0.001).sqrt() + 1e-8)

    sum_fn = None
    red = None
    if push:
        red = parallel.ShardPusher(grads, comm, bucket_bytes=4000)
    if accumulate:
        # two backwards before the step: the arena holds g1, then g1 + g2
        g1 = torch.randn(n, generator=torch.Generator().manual_seed(30 + rank))
        g2 = grads.clone()
        grads.copy_(g1)
        if push:  # the first backward pushes g1's slices
            red.begin(True)
            for upto in (9000, ns - 5, n):
                red.ready(upto)
            red.finish()
        grads += g2
    if overlap or push:
        # backward's arena prefixes become final in uneven steps; buckets of 1000
        # elements (cut at the shard boundaries) are reduced / pushed as they complete
        if push:
            red.begin(not accumulate)
        else:
            red = parallel.GradShardReducer(grads, comm, bucket_bytes=4000)
        for upto in (700, 2500, 2600, 9000, 30001, ns // 2 + 7, ns - 5, n):
            red.ready(upto)
        red.finish()
        if push:
            assert red.consume()
            own, slots = grads[comm.lo:comm.hi], red.slots()

            def sum_fn(out, part):
                x = own.clone()
                for k in range(red.n_slots):  # slot order: the ranks in order, this one left out
                    x += slots[k]
                out.copy_(x)
                sumsq_fn(out, part)
    parallel.zero1_step(comm, grads, gs, partial, sumsq_fn, adam_fn, [p], tail=(ns, n), reduced=overlap,
                        sum_fn=sum_fn)
    for t in (m, v):
        comm.all_gather(t[:ns])  # consolidate
    torch.save({"p": p, "m": m, "v": v}, os.path.join(out_dir, "s%d.pt" % rank))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_optimizer_step_gloo(tmp_path, world):
    """ZeRO-1 orchestration (parallel.ShardComm / zero1_step, the FusedAdam
    sharded path with CPU stand-ins for the two kernels): reduce-scatter, global
    norm from per-shard partial sums, Adam on each shard, all-gather -- equal to
    one process clipping and stepping the summed gradient, at the 2 / 4 / 8 ranks
    of the scaling runs (the arena's ARENA_ALIGN unit splits evenly for each)."""
    mp.spawn(_shard_worker, args=(_port(), str(tmp_path), world), nprocs=world, join=True)
    res = [torch.load(tmp_path / ("s%d.pt" % r), weights_only=True) for r in range(world)]
    r0 = res[0]
    for rr in res[1:]:
        for k in r0:
            torch.testing.assert_close(r0[k], rr[k], rtol=0, atol=0)
    n = 64 * 840 + 192
    p = torch.randn(n, generator=torch.Generator().manual_seed(1))
    gsum = sum(torch.randn(n, generator=torch.Generator().manual_seed(10 + r)) * (r + 1) for r in range(world))
    coef = min(1.0, 2.0 / (float((gsum.double() ** 2).sum()) ** 0.5 + 1e-6))
    gg = gsum * coef + 1e-5 * p
    m, v = 0.1 * gg, 0.001 * gg * gg
    p = p - 1e-3 / 0.1 * m / ((v / 0.001).sqrt() + 1e-8)
    torch.testing.assert_close(r0["p"], p, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(r0["m"], m, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(r0["v"], v, rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize("world,accumulate", [(2, False), (4, False), (2, True)])
def test_pushed_shard_reduce_is_bit_identical_gloo(tmp_path, world, accumulate):
    """NSTL_DP=zero1_push (parallel.ShardPusher, host transport: each rank's
    receive slots a shared /dev/shm mapping, the stand-in for the IPC-mapped
    device buffers the copy engines write): the slices pushed bucket by bucket
    during backward and summed by their owner (own + slots in rank order) give
    the same parameters and moments as the post-backward reduce-scatter -- bit
    for bit at two ranks (one addition either way), to f32 rounding at four.
    With two backwards before the step (gradient accumulation), the second
    push overwrites the first: nothing is counted twice."""
    for push, sub in ((False, "rs"), (True, "push")):
        d = tmp_path / sub
        d.mkdir()
        mp.spawn(_shard_worker, args=(_port(), str(d), world, False, push, accumulate), nprocs=world, join=True)
    for r in range(world):
        a = torch.load(tmp_path / "rs" / ("s%d.pt" % r), weights_only=True)
        b = torch.load(tmp_path / "push" / ("s%d.pt" % r), weights_only=True)
        for k in a:
            if world == 2:
                assert torch.equal(a[k], b[k]), (r, k)
            else:
                torch.testing.assert_close(a[k], b[k], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("world", [2, 4])
def test_overlapped_shard_reduce_is_bit_identical_gloo(tmp_path, world):
    """NSTL_DP=zero1_overlap (parallel.GradShardReducer): the gradient shards
    reduced bucket by bucket onto their owners while backward runs give the same
    parameters and moments as the post-backward reduce-scatter: bit for bit at
    two ranks (one addition either way), to f32 rounding at four (the backend's
    reduce and reduce-scatter may add the four contributions in different
    orders)."""
    for overlap, sub in ((False, "rs"), (True, "ov")):
        d = tmp_path / sub
        d.mkdir()
        mp.spawn(_shard_worker, args=(_port(), str(d), world, overlap), nprocs=world, join=True)
    for r in range(world):
        a = torch.load(tmp_path / "rs" / ("s%d.pt" % r), weights_only=True)
        b = torch.load(tmp_path / "ov" / ("s%d.pt" % r), weights_only=True)
        for k in a:
            if world == 2:
                assert torch.equal(a[k], b[k]), (r, k)
            else:
                torch.testing.assert_close(a[k], b[k], rtol=1e-5, atol=1e-7)


def _reducer_state_worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from neurosync_trainer_lite_amd import parallel
    parallel.init_from_env(backend="gloo")
    ns = 64 * 840
    comm = parallel.ShardComm(ns)
    for cls in (parallel.GradAllReducer, parallel.GradShardReducer):
        g = torch.ones(ns) * (rank + 1)
        red = cls(g, bucket_bytes=4000) if cls is parallel.GradAllReducer else cls(g, comm, bucket_bytes=4000)
        # a completed in-backward reduction is consumed once
        red.begin(True)
        red.ready(ns)
        red.finish()
        assert red.consume() and not red.consume()
        # a backward that raised half-way: the next backward starts from bucket 0
        red.begin(True)
        red.ready(ns // 2)
        assert red.sent > 0 and red.works
        red.begin(True)
        assert red.sent == 0 and not red.works and not red.completed
        # accumulation onto a reduced arena (a second backward before the step) is refused
        red.ready(ns)
        red.finish()
        with pytest.raises(RuntimeError, match="accumulation"):
            red.begin(False)
        # after the step consumed it, accumulation starts a new reduction normally
        red.begin(True)
        red.finish()
        assert red.consume()
        red.begin(False)
    dist.destroy_process_group()


def test_reducer_consume_and_abort_bookkeeping_gloo(tmp_path):
    """the in-backward reducers (NSTL_DP=allreduce / zero1_overlap) mark
    a reduction as done only when finish() completed, the step consumes that
    once (otherwise it reduces itself), a backward that raised leaves no stale
    progress behind, and accumulating a second backward onto already reduced
    gradients raises instead of counting the other ranks' first micro-batch
    twice."""
    mp.spawn(_reducer_state_worker, args=(_port(), str(tmp_path)), nprocs=WORLD, join=True)


def _push_fallback_worker(rank, port, out_dir, world, fail):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from neurosync_trainer_lite_amd import parallel
    parallel.init_from_env(backend="gloo")
    ns = 64 * 840
    comm = parallel.ShardComm(ns)
    g = torch.zeros(comm.numel)
    if fail == "self_test" and rank == world - 1:
        # this rank's markers come out wrong: its peers' checks fail, and so must every rank's setup
        real_push = parallel._HostTransport.push
        parallel._HostTransport.push = lambda self, owner, slot, off, src: real_push(self, owner, slot, off, src * 0 - 7)
    if fail == "setup" and rank == 0:
        parallel.ShardPusher.setup_error = lambda self: RuntimeError("simulated IPC mapping failure")
    red = parallel.ShardPusher.create(g, comm, bucket_bytes=4000)
    # every rank takes the same collectives afterwards, whatever the outcome
    ok = torch.tensor([1.0 if red is not None else 0.0])
    dist.all_reduce(ok)
    torch.save({"made": red is not None, "sum": float(ok)}, os.path.join(out_dir, "f%d.pt" % rank))
    if red is not None:
        red.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,fail", [(2, None), (4, None), (4, "self_test"), (2, "setup")])
def test_push_setup_agrees_on_fallback_gloo(tmp_path, world, fail):
    """ShardPusher.create: the transport is set up, then exercised once (every rank
    pushes a marker into its slot of every peer, then checks its own slots). A
    setup error or a wrong marker on ANY rank makes create() return None on EVERY
    rank (the caller falls back to zero1), with no rank left waiting in a
    collective the others skipped."""
    mp.spawn(_push_fallback_worker, args=(_port(), str(tmp_path), world, fail), nprocs=world, join=True)
    res = [torch.load(tmp_path / ("f%d.pt" % r), weights_only=True) for r in range(world)]
    for r in res:
        assert r["made"] == (fail is None)
        assert r["sum"] == (world if fail is None else 0)


def _push_timeout_worker(rank, port, out_dir, world):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), NSTL_PUSH_TIMEOUT_S="1")
    torch.set_num_threads(1)
    import time
    from neurosync_trainer_lite_amd import parallel
    parallel.init_from_env(backend="gloo")
    comm = parallel.ShardComm(64 * 840)
    # a transport whose copies never complete (a wedged copy engine): every
    # mark stays pending
    parallel._HostTransport.mark = lambda self: [("never", [r for r in range(world) if r != rank])]
    parallel._HostTransport.pending = staticmethod(lambda marks: sorted(r for _, peers in marks for r in peers))
    t0 = time.monotonic()
    try:
        parallel.ShardPusher.create(torch.zeros(comm.numel), comm, bucket_bytes=4000)
        res = "returned"
    except parallel.PushTimeout as e:
        res = str(e)
    torch.save({"res": res, "s": time.monotonic() - t0}, os.path.join(out_dir, "t%d.pt" % rank))
    dist.destroy_process_group()


def test_push_self_test_deadline_raises_gloo(tmp_path):
    """the zero1_push self-test polls its copies from the host
    against the deadline BEFORE anything (stream join, sync, the ranks'
    agreement) is chained behind them, so copies that never land end setup with
    PushTimeout naming the peers, instead of blocking forever; create() does not
    turn it into a zero1 fallback (a copy queue that does not drain cannot be
    trusted by the process)."""
    mp.spawn(_push_timeout_worker, args=(_port(), str(tmp_path), 2), nprocs=2, join=True)
    for r in range(2):
        out = torch.load(tmp_path / ("t%d.pt" % r), weights_only=True)
        assert "not landed after 1 s" in out["res"] and ("[%d]" % (1 - r)) in out["res"], out
        assert out["s"] < 30


def _push_verify_worker(rank, port, out_dir, world, corrupt):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from neurosync_trainer_lite_amd import parallel
    parallel.init_from_env(backend="gloo")
    ns = 64 * 840
    comm = parallel.ShardComm(ns)
    grads = torch.randn(ns, generator=torch.Generator().manual_seed(10 + rank))
    red = parallel.ShardPusher.create(grads, comm, bucket_bytes=4000)
    red.begin(True)
    red.ready(ns)
    red.finish()
    assert red.consume()
    slots = red.slots()
    if corrupt and rank == 0:
        slots[0, 17] += 1.0  # one stale element in one slot of one rank
    gs, part = torch.empty(comm.shard), torch.zeros(4)

    def sumsq_fn(x, p):
        p.zero_()
        p[0] = (x.double() ** 2).sum().float()
    x = grads[comm.lo:comm.hi].clone()
    for k in range(red.n_slots):
        x += slots[k]
    gs.copy_(x)
    sumsq_fn(gs, part)
    ok = red.verify(grads, gs, part, sumsq_fn)
    ref = torch.empty(comm.shard)
    comm.reduce_scatter(grads, ref)
    torch.save({"ok": ok, "failed": red.failed, "check": red.check["ok"], "pending": red.verify_pending,
                "gs_ok": torch.allclose(gs, ref, rtol=1e-6, atol=1e-6),
                "part_ok": abs(float(part[0]) - float((ref.double() ** 2).sum())) <= 1e-3 * float(part[0])},
               os.path.join(out_dir, "v%d.pt" % rank))
    red.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,corrupt", [(2, False), (4, False), (4, True)])
def test_push_first_step_verified_against_reduce_scatter_gloo(tmp_path, world, corrupt):
    """the first step's pushed shard sums (own + slots) are checked
    against the reduce-scatter of the same arena, on every rank, and the ranks
    agree: one stale element on one rank fails the check everywhere; that step
    then continues on the reduce-scatter's shard and sums of squares, and the
    reducer is marked failed (the optimizer runs zero1 from then on)."""
    mp.spawn(_push_verify_worker, args=(_port(), str(tmp_path), world, corrupt), nprocs=world, join=True)
    for r in range(world):
        out = torch.load(tmp_path / ("v%d.pt" % r), weights_only=True)
        assert out["ok"] == out["check"] == (not corrupt), out
        assert out["failed"] == corrupt and out["pending"] is False
        assert out["gs_ok"] and out["part_ok"], out
