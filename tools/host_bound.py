"""Is the 228M step host-bound?  Per step: the host time to enqueue it (the
step() call returns before the GPU runs it) and the GPU time between two
events around it, first with the queue drained before each step (host and
device time measured apart), then back to back (the bench's regime).
  python tools/host_bound.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd.config import training_config  # noqa: E402
from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components  # noqa: E402

dev = torch.device("cuda", 0)
cfg = dict(training_config)
cfg.update(micro_batch_size=128, frame_size=128, batch_size=128)
torch.manual_seed(0)
model = build_model(cfg, dev)
model.train()
crit, opt, _ = prepare_training_components(cfg, model)
opt.trust_backward_norm = True
src = torch.randn(128, 128, 256, device=dev)
trg = torch.randn(128, 128, 61, device=dev) * 20


def step():
    opt.zero_grad()
    crit(model(src), trg).backward()
    opt.step(max_norm=2.0)


for _ in range(5):
    step()
torch.cuda.synchronize()
host, gpu = [], []
for _ in range(10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    t0 = time.perf_counter()
    step()
    host.append((time.perf_counter() - t0) * 1e3)
    e1.record()
    torch.cuda.synchronize()
    gpu.append(e0.elapsed_time(e1))
host.sort()
gpu.sort()
print("drained queue: host enqueue %.2f ms/step (median), GPU %.2f ms/step (median)" % (host[5], gpu[5]))
n = 20
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    step()
t_host = (time.perf_counter() - t0) / n * 1e3
torch.cuda.synchronize()
t_all = (time.perf_counter() - t0) / n * 1e3
print("back to back: host returns after %.2f ms/step, wall %.2f ms/step" % (t_host, t_all))
