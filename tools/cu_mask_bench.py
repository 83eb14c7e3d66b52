"""Step time of the 228M training step on a compute stream that excludes k CUs
(hipExtStreamCreateWithCUMask): what ceding CUs to RCCL's channel workgroups
during backward costs the step (NSTL_DP=zero1_overlap).
Mask bit i is a CU of XCD i % 8 (tools/micro/cu_probe.hip); pattern "first"
(default) clears bits 0 .. k-1, i.e. ceil(k / 8) CUs on the first min(k, 8)
XCDs -- one per XCD at k = 8.  The persistent grids take 8 x the fewest CUs left
on one XCD (nstl_stream_cus) and the GEMM deals what does not divide into them
stream-K.  "spread" clears one bit per 256 / k: all of them on XCD 0 (the
round-3 table's pattern).
  python tools/cu_mask_bench.py [k ...] [--pattern first|spread|last]"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def masked_stream(dev, n_cus, excluded):
    """A HIP stream of the runtime torch uses, restricted to the CUs not in `excluded`."""
    hip = ctypes.CDLL(os.path.join(HERE, "neurosync_trainer_lite_amd", "libnstl_hip.so"))
    fn = hip.hipExtStreamCreateWithCUMask
    fn.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    words = (n_cus + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in range(n_cus):
        if c not in excluded:
            mask[c // 32] |= 1 << (c % 32)
    st = ctypes.c_void_p()
    rc = fn(ctypes.byref(st), words, mask)
    if rc != 0:
        raise RuntimeError("hipExtStreamCreateWithCUMask failed: %d" % rc)
    return torch.cuda.ExternalStream(st.value, device=dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ks", nargs="*", type=int, default=[0, 2, 4, 8, 16, 32])
    ap.add_argument("--steps", type=int, default=15)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--pattern", default="first", choices=["spread", "first", "last"],
                    help="which mask bits are cleared: one per n/k (spread), the first k, or the last k")
    args = ap.parse_args()
    from neurosync_trainer_lite_amd.config import training_config
    from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components
    dev = torch.device("cuda", 0)
    n_cus = torch.cuda.get_device_properties(0).multi_processor_count
    cfg = dict(training_config)
    cfg.update(micro_batch_size=128, frame_size=128, batch_size=128)
    torch.manual_seed(0)
    model = build_model(cfg, dev)
    model.train()
    crit, opt, _ = prepare_training_components(cfg, model)
    opt.trust_backward_norm = True
    src = torch.randn(128, 128, 256, device=dev)
    trg = torch.randn(128, 128, 61, device=dev) * 20
    streams = {}
    for k in args.ks:
        if k == 0:
            ex = set()
        elif args.pattern == "spread":
            ex = {(i * n_cus) // k for i in range(k)}
        elif args.pattern == "first":
            ex = set(range(k))
        else:
            ex = set(range(n_cus - k, n_cus))
        streams[k] = masked_stream(dev, n_cus, ex)

    def step():
        opt.zero_grad()
        crit(model(src), trg).backward()
        opt.step(max_norm=2.0)

    rows = {}
    for rep in range(args.reps):
        for k in args.ks:
            s = streams[k]
            torch.cuda.synchronize()
            with torch.cuda.stream(s):
                for _ in range(3):
                    step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    step()
                torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.steps * 1e3
            rows.setdefault(k, []).append(ms)
            print("k=%2d excluded CUs: %.3f ms/step" % (k, ms), flush=True)
    base = min(rows[0]) if 0 in rows else None
    out = {"n_cus": n_cus, "steps": args.steps, "pattern": args.pattern,
           "ms_per_step": {k: round(min(v), 3) for k, v in rows.items()},
           "cost_ms": {k: round(min(v) - base, 3) for k, v in rows.items()} if base else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
