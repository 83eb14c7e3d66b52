"""RCCL beside the backward on one GPU: the 228M bench step (B=128, T=128) in a
world_size-1 RCCL group, with the bucketed gradient all-reduce (NSTL_DP=allreduce,
64 MB buckets launched as backward completes them) forced on, against the same
step without it.  Run under rocprofv3 --kernel-trace to see whether RCCL puts a
kernel on the device for one rank (it decides per call).  Channel limits come
from NCCL_MIN_NCHANNELS / NCCL_MAX_NCHANNELS in the environment.
  python tools/rccl_probe.py [steps]"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import parallel  # noqa: E402
from neurosync_trainer_lite_amd.config import training_config  # noqa: E402
from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29611")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
cfg = dict(training_config)
torch.manual_seed(0)
model = build_model(cfg, "cuda:0")
crit, opt, _ = prepare_training_components(cfg, model)
model.train()
g = torch.Generator(device="cuda:0").manual_seed(1)
src = torch.randn(128, 128, 256, device="cuda:0", generator=g)
trg = torch.randn(128, 128, 61, device="cuda:0", generator=g) * 20
eng = None


def run(n):
    for _ in range(n):
        opt.zero_grad()
        crit(model(src), trg).backward()
        opt.step(max_norm=2.0)


res = {"NCCL_MIN_NCHANNELS": os.environ.get("NCCL_MIN_NCHANNELS"),
       "NCCL_MAX_NCHANNELS": os.environ.get("NCCL_MAX_NCHANNELS")}
run(3)
eng = model.engine()
for arm in ("plain", "allreduce", "plain", "allreduce"):
    eng.grad_reducer = parallel.GradAllReducer(eng.g32, min_world=1) if arm == "allreduce" else None
    run(2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    res.setdefault(arm, []).append(round(ms, 3))
    print(arm, "%.3f ms/step" % ms, flush=True)
print(json.dumps(res))
dist.destroy_process_group()
