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


if __name__ == "__main__":
    main()
