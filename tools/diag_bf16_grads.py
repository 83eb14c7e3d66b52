"""Diagnostic: per-tensor gradient error of the bf16 step at production shape
(B=128, T=128, D=1024, H=16, L=4) against the fp32 oracle, beside the error of
the reference model itself run under torch bf16 autocast on the GPU (what the
reference's own mixed precision gives).  Prints the worst tensors of each."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import model_ref  # noqa: E402
from tests.test_production_gpu import D, H, L, B, T, rel, run_step  # noqa: E402

params = model_ref.seeded_params(model_ref.param_shapes(256, D, L, 61), 61)
rng = np.random.default_rng(62)
src = torch.tensor(rng.standard_normal((B, T, 256)).astype(np.float32))
trg = torch.tensor((rng.standard_normal((B, T, 61)) * 20).astype(np.float32))
t0 = time.time()
o = model_ref.OracleTrainer(params, H)
o_loss, o_norm, o_pred = o.step(src, trg)
print("oracle %.1fs loss %.6f norm %.6f" % (time.time() - t0, o_loss.item(), o_norm.item()), flush=True)
og = o.last_grads

pred, loss, norm, grads, c = run_step(params, src, trg, amp=True)
print("ours bf16: loss %.6f norm %.6f rel(pred) %.3e" % (loss, norm, rel(pred, o_pred)))

# reference under autocast(bf16) on the GPU
p = {k: v.detach().clone().cuda().requires_grad_(True) for k, v in params.items()}
with torch.autocast("cuda", dtype=torch.bfloat16):
    ap = model_ref.seq2seq_forward(p, src.cuda(), H)
    al = model_ref.loss_fn(ap.float(), trg.cuda())
al.backward()
ag = {k: v.grad.detach().cpu() for k, v in p.items()}
print("ref autocast bf16: loss %.6f rel(pred) %.3e" % (al.item(), rel(ap.detach().float(), o_pred)))
rows = sorted(((rel(grads[k], og[k]), rel(ag[k], og[k]), og[k].norm().item(), k) for k in og), reverse=True)
print("%-62s %9s %9s %10s" % ("tensor", "ours", "autocast", "|g|"))
for r in rows[:25]:
    print("%-62s %9.3e %9.3e %10.3e" % (r[3], r[0], r[1], r[2]))
print("max ours %.3e  max autocast %.3e  max ratio %.2f" % (
    max(r[0] for r in rows), max(r[1] for r in rows), max(r[0] / max(r[1], 1e-12) for r in rows)))

# fp32: ours (parity mode) and the oracle's own fp32 on the GPU, against the CPU oracle
pred32, loss32, norm32, grads32, c32 = run_step(params, src, trg, amp=False)
p = {k: v.detach().clone().cuda().requires_grad_(True) for k, v in params.items()}
gp = model_ref.seq2seq_forward(p, src.cuda(), H)
model_ref.loss_fn(gp, trg.cuda()).backward()
gg = {k: v.grad.detach().cpu() for k, v in p.items()}
print("fp32: ours rel(pred) %.3e, torch-gpu rel(pred) %.3e" % (rel(pred32, o_pred), rel(gp.detach(), o_pred)))
rows = sorted(((rel(grads32[k], og[k]), rel(gg[k], og[k]), og[k].norm().item(), k) for k in og), reverse=True)
print("%-62s %9s %9s %10s" % ("tensor", "ours32", "torchgpu", "|g|"))
for r in rows[:25]:
    print("%-62s %9.3e %9.3e %10.3e" % (r[3], r[0], r[1], r[2]))
