"""Host-side cost of the 228M training step: how long the Python/ctypes/HIP
launch path takes to enqueue one step (no synchronisation inside) against the
GPU time of the step.  When the enqueue time approaches the GPU time the GPU
starves between kernels.  Also times each phase's enqueue (forward, loss,
backward, optimizer) with the queue kept short by a sync before each phase.
  python tools/host_time.py [--steps N]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    from neurosync_trainer_lite_amd.config import training_config
    from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components
    dev = torch.device("cuda", 0)
    cfg = dict(training_config, micro_batch_size=128, frame_size=128, batch_size=128)
    torch.manual_seed(1234)
    model = build_model(cfg, dev)
    model.train()
    crit, opt, _ = prepare_training_components(cfg, model)
    opt.trust_backward_norm = True
    g = torch.Generator(device=dev).manual_seed(100)
    src = torch.randn(128, 128, cfg["input_dim"], device=dev, generator=g)
    trg = torch.randn(128, 128, cfg["output_dim"], device=dev, generator=g) * 20
    for _ in range(3):
        opt.zero_grad()
        loss = crit(model(src), trg)
        loss.backward()
        opt.step(max_norm=2.0)
    torch.cuda.synchronize()
    # whole steps back to back: host enqueue time per step vs wall per step
    host = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        h0 = time.perf_counter()
        opt.zero_grad()
        loss = crit(model(src), trg)
        loss.backward()
        opt.step(max_norm=2.0)
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    print("back to back: wall %.2f ms/step, host enqueue %.2f ms/step (min %.2f)" %
          (wall * 1e3, sum(host) / len(host) * 1e3, min(host) * 1e3))
    # per phase, each starting from an idle GPU (host time only, then the GPU time)
    ph = {"fwd+loss": [], "bwd": [], "opt": []}
    gpu = {"fwd+loss": [], "bwd": [], "opt": []}
    for _ in range(a.steps):
        opt.zero_grad()
        torch.cuda.synchronize()
        for name, fn in (("fwd+loss", lambda: crit(model(src), trg)),):
            h0 = time.perf_counter()
            loss = fn()
            ph[name].append(time.perf_counter() - h0)
            torch.cuda.synchronize()
            gpu[name].append(time.perf_counter() - h0)
        h0 = time.perf_counter()
        loss.backward()
        ph["bwd"].append(time.perf_counter() - h0)
        torch.cuda.synchronize()
        gpu["bwd"].append(time.perf_counter() - h0)
        h0 = time.perf_counter()
        opt.step(max_norm=2.0)
        ph["opt"].append(time.perf_counter() - h0)
        torch.cuda.synchronize()
        gpu["opt"].append(time.perf_counter() - h0)
    for k in ph:
        print("%-9s host enqueue %.2f ms, host+GPU %.2f ms" % (k, sum(ph[k]) / len(ph[k]) * 1e3,
                                                            sum(gpu[k]) / len(gpu[k]) * 1e3))


if __name__ == "__main__":
    main()
