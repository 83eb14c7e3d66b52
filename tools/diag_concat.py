"""Diagnostic: the NSTL_DMEM_CONCAT 1-vs-0 gradient difference of
tests/test_model_gpu.py::test_bf16_concatenated_memory_gradient_matches_per_layer,
and the run-to-run difference of one arm (determinism check)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_model_gpu import make, rel, DEV  # noqa: E402


def grads(cat, dropout):
    os.environ["NSTL_DMEM_CONCAT"] = cat
    cfg, model, crit, opt, params = make(256, 4, 3, 11, amp=True, dropout=dropout)
    torch.manual_seed(5)
    g = torch.Generator().manual_seed(6)
    src = torch.randn(4, 128, 256, generator=g).to(DEV)
    trg = (torch.randn(4, 128, 61, generator=g) * 20).to(DEV)
    model.train()
    opt.zero_grad()
    crit(model(src), trg).backward()
    torch.cuda.synchronize()
    return {k: p.grad.detach().double().cpu().clone() for k, p in model.named_parameters()}


for dropout in (0.1, 0.0):
    a, a2, b = grads("1", dropout), grads("1", dropout), grads("0", dropout)
    print("dropout", dropout, "concat vs per-layer worst %.3e" % max(rel(a[k], b[k]) for k in a),
          " rerun worst %.3e" % max(rel(a[k], a2[k]) for k in a))
