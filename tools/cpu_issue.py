"""Host issue time of one training step vs its GPU time (228M, B=128, T=128).
If the host needs as long as the GPU, the step is launch-bound."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd.config import training_config  # noqa: E402
from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components  # noqa: E402

dev = torch.device("cuda", 0)
cfg = dict(training_config)
B, T = 128, 128
cfg.update(micro_batch_size=T, frame_size=T, batch_size=B)
torch.manual_seed(0)
model = build_model(cfg, dev)
model.train()
crit, opt, _ = prepare_training_components(cfg, model)
src = torch.randn(B, T, cfg["input_dim"], device=dev)
trg = torch.randn(B, T, cfg["output_dim"], device=dev)


def step():
    opt.zero_grad()
    loss = crit(model(src), trg)
    loss.backward()
    opt.step(max_norm=2.0)


for _ in range(3):
    step()
torch.cuda.synchronize()
# host time per phase with the GPU idle at the start (queue empty)
t0 = time.perf_counter()
opt.zero_grad()
out = model(src)
t1 = time.perf_counter()
loss = crit(out, trg)
t2 = time.perf_counter()
loss.backward()
t3 = time.perf_counter()
opt.step(max_norm=2.0)
t4 = time.perf_counter()
torch.cuda.synchronize()
t5 = time.perf_counter()
print("host issue: fwd %.2f ms  loss %.2f  bwd %.2f  opt %.2f  (total %.2f)  -> GPU drained at %.2f ms" % (
    (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3, (t4 - t0) * 1e3, (t5 - t0) * 1e3))
n = 10
t0 = time.perf_counter()
for _ in range(n):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("%d steps: host issue %.2f ms/step, wall %.2f ms/step" % (n, (t1 - t0) / n * 1e3, (t2 - t0) / n * 1e3))
