"""What the copy-engine ZeRO-1 push (NSTL_DP=zero1_push, parallel.ShardPusher)
costs the step it runs beside, measured on one GPU.

At n ranks a rank pushes (n-1)/n of its f32 gradient arena to the owners during
backward (at n = 8: 824 MB of the 942 MB arena at the 228M shape) and receives
as much; on its own HBM that is the same bytes read (its pushes) and written
(the pushes it receives).  This tool reproduces exactly that local traffic with
the real mechanism: a stand-in reducer on the engine (the ShardPusher
interface: begin / ready / finish) copies (n-1)/n of every final arena bucket
into a device buffer with nstl_copy_engine (hipMemcpyDeviceToDeviceNoCU: copy
engines, no kernel) -- on NSTL_PUSH_STREAMS streams as _DeviceTransport does
(--streams k: k streams), the bucket's part cut in one slice per stream -- at the points of backward where
ShardPusher would push, and the step waits for the copies before its optimizer
(as ShardPusher.finish does).  The step time is compared with the same step
without the copies, in alternating blocks.  A kernel trace of the run
(rocprofv3 --kernel-trace) shows whether any copy kernel ran
(`__amd_rocclr_copyBuffer`): none should.

  python tools/copy_interference.py [--ranks 8] [--steps 20] [--reps 3]

--exchange: the WHOLE exchange of one rank at n ranks, not
just the pushes.  Arm "n1" is the 1-GPU step (clip + Adam over every
parameter).  Arm "stand-in" is one rank's step at n ranks with every local
byte the exchange moves: the pushes during backward (above; their local
destination buffer stands in for the slots this rank receives), then
nstl_shard_sum over own + the (n-1) slots (the clip norm's partials in the same
pass), the sharded Adam on 1/n of the matrices (+ the replicated f32 tail, with
its own sums of squares), then the copy-engine all-gather of the updated bf16
shard to (n-1) peers (one stream per peer, as _DeviceTransport.gather; here
into a local buffer, which stands in for both the bytes sent and the bytes the
peers write into this rank's arena).  What one GPU cannot show: the
collectives' latency (two 4-byte syncs and a 4 KB all-reduce), xGMI link
rates above the copy engines' local rate, and the ranks' skew.  Reported per
arm: ms per step, and the post-backward segment (backward's end to the next
forward's first kernel, HIP events on the compute stream).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class CopyProbe:
    """Pushes (n-1)/n of each 64 MB bucket of the final arena prefix with the copy
    engines, as ShardPusher would at n ranks (inactive for the optimizer)."""

    active = False  # FusedAdam: no reduction to consume

    def __init__(self, K, g, ranks, bucket_bytes=64 << 20, streams=None):
        self.K, self.g = K, g
        self.frac = (ranks - 1) / ranks
        self.bucket = bucket_bytes // 4
        self.dst = torch.empty(int(g.numel() * self.frac) + self.bucket, dtype=torch.float32, device=g.device)
        if not streams:
            from neurosync_trainer_lite_amd.parallel import push_streams
            streams = min(push_streams(), ranks - 1)
        self.sides = [torch.cuda.Stream(g.device) for _ in range(max(1, streams))]
        self.sent = 0
        self.out = 0
        self.bytes = 0

    def begin(self, fresh):
        self.sent = self.out = 0

    def _push(self, lo, hi):
        n = int((hi - lo) * self.frac)
        if n <= 0:
            return
        # the bucket's pushed part as one slice per owner, each on that owner's stream
        ns = len(self.sides)
        cut = [lo + (n * i) // ns for i in range(ns + 1)]
        for i, side in enumerate(self.sides):
            a, b = cut[i], cut[i + 1]
            if b <= a:
                continue
            side.wait_stream(torch.cuda.current_stream())
            self.K.copy_engine(self.dst[self.out + a - lo:].data_ptr(), self.g[a:b], (b - a) * 4,
                               stream=side.cuda_stream)
        self.out += n
        self.bytes += n * 4

    def ready(self, upto):
        while upto - self.sent >= self.bucket:
            self._push(self.sent, self.sent + self.bucket)
            self.sent += self.bucket

    def finish(self):
        if self.sent < self.g.numel():
            self._push(self.sent, self.g.numel())
            self.sent = self.g.numel()
        for side in self.sides:
            torch.cuda.current_stream().wait_stream(side)

    def consume(self):
        return False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--streams", type=int, default=0, help="copy streams (default NSTL_PUSH_STREAMS, as the product)")
    ap.add_argument("--trace-only", action="store_true", help="a few steps with the copies (for a kernel trace)")
    ap.add_argument("--exchange", action="store_true", help="the whole exchange at --ranks (see the module doc)")
    args = ap.parse_args()
    from neurosync_trainer_lite_amd import _hip as K
    from neurosync_trainer_lite_amd.config import training_config
    from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components
    dev = torch.device("cuda", 0)
    cfg = dict(training_config)
    B, T = 128, 128
    cfg.update(micro_batch_size=T, frame_size=T, batch_size=B)
    torch.manual_seed(1234)
    model = build_model(cfg, dev)
    model.train()
    crit, opt, _ = prepare_training_components(cfg, model)
    eng = model.engine()
    g = torch.Generator(device=dev).manual_seed(100)
    src = torch.randn(B, T, cfg["input_dim"], device=dev, generator=g)
    trg = torch.randn(B, T, cfg["output_dim"], device=dev, generator=g) * 20

    def step():
        opt.zero_grad()
        crit(model(src), trg).backward()
        opt.step(max_norm=2.0)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    probe = CopyProbe(K, eng.g32, args.ranks, streams=args.streams or None)
    if args.exchange:
        return exchange(args, K, model, crit, opt, eng, src, trg, probe)

    def block(with_copies, steps):
        eng.grad_reducer = probe if with_copies else None
        probe.bytes = 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        eng.grad_reducer = None
        return ms, probe.bytes / steps

    if args.trace_only:
        block(True, 5)
        return
    rows = []
    for rep in range(args.reps):
        for arm in ((False, True) if rep % 2 == 0 else (True, False)):
            ms, by = block(arm, args.steps)
            rows.append({"rep": rep, "copies": arm, "ms_per_step": round(ms, 3), "copied_MB_per_step": round(by / 1e6, 1)})
            print(json.dumps(rows[-1]), flush=True)
    base = [r["ms_per_step"] for r in rows if not r["copies"]]
    cop = [r["ms_per_step"] for r in rows if r["copies"]]
    mb = sum(base) / len(base)
    mc = sum(cop) / len(cop)
    print(json.dumps({"ranks": args.ranks, "streams": len(probe.sides), "ms_without": round(mb, 3), "ms_with_copies": round(mc, 3),
                      "cost_pct": round((mc / mb - 1) * 100, 2), "copied_MB_per_step": rows[-1]["copied_MB_per_step"]}))


def exchange(args, K, model, crit, opt, eng, src, trg, probe):
    n = args.ranks
    opt.trust_backward_norm = True  # as bench.py's 1-GPU step
    shard = eng.n_shardable // n
    lo, hi = 0, shard  # rank 0's shard
    assert probe.dst.numel() >= (n - 1) * shard
    slots = probe.dst[:(n - 1) * shard].view(n - 1, shard)
    gs = torch.empty(shard, dtype=torch.float32, device=eng.device)
    partial = torch.zeros(1024, dtype=torch.float32, device=eng.device)
    part_t = torch.zeros(1024, dtype=torch.float32, device=eng.device)
    norm = torch.zeros(1, dtype=torch.float32, device=eng.device)
    gat = torch.empty((n - 1) * shard, dtype=eng.p16.dtype, device=eng.device)
    gsides = [torch.cuda.Stream(eng.device) for _ in range(n - 1)]
    grp = opt.param_groups[0]

    def adam(a_lo, cnt, grads, part):
        a = K.AdamArgs()
        a.lowp_dtype = K.dtype_code(eng.p16.dtype)
        a.lr, a.eps, a.weight_decay = grp["lr"], grp["eps"], grp["weight_decay"]
        a.beta1, a.beta2 = grp["betas"]
        a.step = 1
        a.sumsq_partial, a.n_partial, a.max_norm, a.norm_out = part.data_ptr(), 1024, 2.0, norm.data_ptr()
        a.p, a.g, a.m, a.v = (eng.p32[a_lo:].data_ptr(), grads.data_ptr(), opt.m[a_lo:].data_ptr(),
                              opt.v[a_lo:].data_ptr())
        a.p_lowp = eng.p16[a_lo:].data_ptr()
        a.n = cnt
        K.adam_step(a)

    def sharded_update():
        K.shard_sum(eng.g32[lo:hi], slots, n - 1, gs, partial, 1024)
        t_lo, t_hi = eng.n_shardable, eng.numel  # the replicated f32 tail
        K.sumsq(eng.g32[t_lo:t_hi], t_hi - t_lo, part_t, 1024)
        partial.add_(part_t)
        adam(t_lo, t_hi - t_lo, eng.g32[t_lo:t_hi], partial)
        adam(lo, shard, gs, partial)
        cur = torch.cuda.current_stream()
        for i, st in enumerate(gsides):
            st.wait_stream(cur)
            K.copy_engine(gat[i * shard:].data_ptr(), eng.p16[lo:hi], shard * eng.p16.element_size(),
                          stream=st.cuda_stream)
        for st in gsides:
            cur.wait_stream(st)

    evs = []

    def step(stand_in):
        opt.zero_grad()
        crit(model(src), trg).backward()
        e1, e2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e1.record()
        if stand_in:
            eng.sync_pending()
            sharded_update()
        else:
            opt.step(max_norm=2.0)
        e2.record()
        evs.append((e1, e2))

    def block(stand_in, steps):
        eng.grad_reducer = probe if stand_in else None
        probe.bytes = 0
        evs.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step(stand_in)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        eng.grad_reducer = None
        post = sorted(a.elapsed_time(b) for a, b in evs)[len(evs) // 2]
        return ms, post, probe.bytes / steps

    block(True, 3)
    rows = []
    for rep in range(args.reps):
        for arm in ((False, True) if rep % 2 == 0 else (True, False)):
            ms, post, by = block(arm, args.steps)
            rows.append({"rep": rep, "arm": "stand-in" if arm else "n1", "ms_per_step": round(ms, 3),
                         "post_backward_ms_median": round(post, 3), "pushed_MB_per_step": round(by / 1e6, 1)})
            print(json.dumps(rows[-1]), flush=True)

    def mean(arm, k):
        v = [r[k] for r in rows if r["arm"] == arm]
        return round(sum(v) / len(v), 3)
    esz = eng.p16.element_size()
    print(json.dumps({"ranks": n, "shard_elems": shard, "push_streams": len(probe.sides),
                      "ms_n1": mean("n1", "ms_per_step"), "ms_stand_in": mean("stand-in", "ms_per_step"),
                      "post_backward_ms_n1": mean("n1", "post_backward_ms_median"),
                      "post_backward_ms_stand_in": mean("stand-in", "post_backward_ms_median"),
                      "bytes": {"pushed_during_backward_MB": max(r["pushed_MB_per_step"] for r in rows),
                                "shard_sum_read_MB": round(n * shard * 4 / 1e6, 1),
                                "gather_out_MB": round((n - 1) * shard * esz / 1e6, 1)}}))


if __name__ == "__main__":
    main()
