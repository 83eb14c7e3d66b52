"""Step time of the 228M training step while `nblocks` workgroups (each with
`lds` bytes of LDS, like an RCCL all-reduce channel) hold CUs on a side stream:
how sensitive the 1-workgroup-per-CU kernels are to sharing the chip.
  python tools/cu_hog_bench.py [nblocks ...]"""
import ctypes
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from neurosync_trainer_lite_amd.config import training_config  # noqa: E402
from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components  # noqa: E402

hog = ctypes.CDLL(os.path.join(HERE, "tools", "micro", "libcuhog.so"))
hog.cu_hog.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p]
dev = torch.device("cuda", 0)
cfg = dict(training_config)
cfg.update(micro_batch_size=128, frame_size=128, batch_size=128)
torch.manual_seed(0)
model = build_model(cfg, dev)
model.train()
crit, opt, _ = prepare_training_components(cfg, model)
src = torch.randn(128, 128, 256, device=dev)
trg = torch.randn(128, 128, 61, device=dev)
side = torch.cuda.Stream(dev)


def step():
    opt.zero_grad()
    crit(model(src), trg).backward()
    opt.step(max_norm=2.0)


for _ in range(3):
    step()
torch.cuda.synchronize()
for nb in [int(a) for a in sys.argv[1:]] or [0, 8, 16, 32]:
    steps = 10
    if nb:
        # hold the CUs for longer than the timed steps
        hog.cu_hog(nb, 8192, 150_000_000, side.cuda_stream)  # 1.5 s at 100 MHz
        time.sleep(0.05)
    torch.cuda.synchronize(dev) if not nb else None
    t0 = time.perf_counter()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(steps):
        step()
    ev1.record()
    ev1.synchronize()
    ms = ev0.elapsed_time(ev1) / steps
    print("hog %3d workgroups: %.2f ms/step" % (nb, ms), flush=True)
    if nb:
        torch.cuda.synchronize()  # wait for the hog to finish
