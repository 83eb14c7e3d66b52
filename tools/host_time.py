"""Host-side cost of the 228M step: how long Python takes to issue one step (the
GPU queue absorbs the launches, so this is hidden while it stays below the GPU
step time), and the part of it spent in the argument extent checks
(_hip.gemm_check / _need / attn_set ...), by cProfile over a few steps.
  python tools/host_time.py"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
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
    host, gpu = [], []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append(t1 - t0)
        gpu.append(t2 - t0)
    host.sort()
    gpu.sort()
    print("host issue time per step %.2f ms (median of 10), step with sync %.2f ms" % (host[5] * 1e3, gpu[5] * 1e3))
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    pr.enable()
    for _ in range(5):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    tot = 0.0
    for (fn, line, name), (cc, nc, tt, ct, callers) in st.stats.items():
        if name in ("gemm_check", "_need", "_need_mat", "_check_side", "_room") and "_hip" in fn:
            if name == "gemm_check":
                print("gemm_check: %d calls per step, %.3f ms per step (cumulative)" % (nc // 5, ct / 5 * 1e3))
            if name == "_need":
                tot = ct / 5
                print("_need (every extent check): %d calls per step, %.3f ms per step" % (nc // 5, tot * 1e3))


if __name__ == "__main__":
    main()
