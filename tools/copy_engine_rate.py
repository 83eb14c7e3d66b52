"""Copy-engine rate on one GPU: the bf16 weight all-gather of zero1_push at 8
ranks moves 7 slices of one rank's shard (59 MB each at the 228M shape) with
nstl_copy_engine (hipMemcpyDeviceToDeviceNoCU), one stream per peer.  Here the
seven copies go device to device on one GPU, on 1 and on 7 streams, to show
whether the engines run concurrently (the xGMI rate itself needs the 8-GPU node).
  python tools/copy_engine_rate.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402

dev = torch.device("cuda", 0)
SLICE = 59 * (1 << 20) // 2  # bf16 elements
src = torch.randn(SLICE, device=dev).to(torch.bfloat16)
dst = [torch.empty(SLICE, dtype=torch.bfloat16, device=dev) for _ in range(7)]
for n_streams in (1, 7, 1, 7):
    streams = [torch.cuda.Stream(dev) for _ in range(n_streams)]
    for rep in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, d in enumerate(dst):
            s = streams[i % n_streams]
            K.copy_engine(d.data_ptr(), src, SLICE * 2, stream=s.cuda_stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print("7 x 59 MB on %d stream(s): %.2f ms, %.1f GB/s" % (n_streams, dt * 1e3, 7 * SLICE * 2 / dt / 1e9), flush=True)
