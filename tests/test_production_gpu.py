"""Production-shape parity: the training step at B*T = 16,384 frames (B=128
windows x T=128, D=1024, H=16) against the CPU oracle, through the kernels the
228M bench runs (reference step: utils/training_utils.py:56-80).

At this shape the bf16 step takes the 256x256 LDS-DMA ring GEMM for every
projection, the grouped weight-gradient launches (one 256-tile launch per
decoder layer, one 768-tile launch per 4 encoder layers), the fused attention
backward over B*H = 2,048 (b, h) blocks and the batched row reductions; the
launch counters of the C ABI (nstl_kernel_counts) assert that choice.  L=4 is
the smallest depth with a full 4-layer encoder group.

Bounds are those of tests/test_model_gpu.py (fp32: forward 1e-4, gradients 1e-4
relative per tensor; bf16: forward 3e-2, loss 2e-2, gradients 0.1), plus the
metric's forward MSE gate (1e-3).

fp32 gradients: run against the unmodified oracle, every gradient differs by
~1.2e-3 relative while the forward agrees to 1.3e-6 -- and the reference's own
code run by torch in fp32 on the GPU differs from the CPU run by the same
~1.1e-3, with the loss's direction term on or off.  The cause is the FFN ReLU:
of the 2 x 4 x 67 M pre-activations of an L=4 step, ~700 lie within 1e-6 of
zero and ~180 land on the other side of it in the oracle than in our kernels
(f32 summation order), and each flip passes or blocks a gradient row.  So the
unpinned fp32 check keeps the floor max(1e-4, 2 x the torch-GPU fp32 error),
and test_fp32_production_step_relu_pinned pins the oracle's ReLU pattern to
our forward's: every gradient then agrees to 5e-6 (bound 1e-4, no floor).

bf16 gradients: the reference's own mixed precision (the oracle model under
torch bf16 autocast on the GPU) already misses the fp32 gradients by up to 0.11
relative on some tensors (tiny-norm, cancellation-dominated ones such as the q
biases, and the deepest encoder weights: tools/diag_bf16_grads.py), so with the
reference loss a tensor passes at max(0.1, 1.5 x that autocast error); with the
direction term off (w3 = 0) every tensor is held to 0.1 with no floor.
"""
import time

import numpy as np
import pytest
import torch

from neurosync_trainer_lite_amd import _hip as K
from oracle import model_ref

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
D, H, L, B, T = 1024, 16, 4, 128, 128


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def make_problem(n_layers, seed, w3):
    params = model_ref.seeded_params(model_ref.param_shapes(256, D, n_layers, 61), seed)
    rng = np.random.default_rng(seed + 1)
    src = torch.tensor(rng.standard_normal((B, T, 256)).astype(np.float32))
    trg = torch.tensor((rng.standard_normal((B, T, 61)) * 20).astype(np.float32))
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    t0 = time.time()
    oracle = model_ref.OracleTrainer(params, H, w3=w3)
    o_loss, o_norm, o_pred = oracle.step(src, trg)
    print("oracle step (L=%d, w3=%g) %.1f s" % (n_layers, w3, time.time() - t0))
    return params, src, trg, o_loss, o_norm, o_pred, oracle.last_grads


@pytest.fixture(scope="module")
def problem():
    return make_problem(L, 61, 1.0)


@pytest.fixture(scope="module")
def problem_w3_0():
    """The same shape with the loss's direction term off (w3 = 0: Huber + L1 of
    first differences, utils/model.py:278-291 with w3 = 0)."""
    return make_problem(L, 61, 0.0)


def run_step(params, src, trg, amp, w3=1.0, n_layers=L, want_model=False, fp8=False):
    from neurosync_trainer_lite_amd.config import training_config
    from neurosync_trainer_lite_amd.utils.model import Loss
    from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components
    cfg = dict(training_config)
    cfg.update(hidden_dim=D, num_heads=H, n_layers=n_layers, dropout=0.0, use_amp=amp)
    model = build_model(cfg, DEV)
    model.load_state_dict(params, strict=True)
    if fp8:
        model.set_fp8(True, backward=True)
    crit, opt, _ = prepare_training_components(cfg, model)
    if w3 != 1.0:
        crit = Loss(1.0, 1.0, 1.0, w3)
    model.train()
    opt.zero_grad()
    pred = model(src.to(DEV))  # builds the workspace; the counted step follows
    torch.cuda.synchronize()
    K.kernel_counts_reset()
    opt.zero_grad()
    pred = model(src.to(DEV))
    loss = crit(pred, trg.to(DEV))
    loss.backward()
    opt.step(max_norm=2.0)
    torch.cuda.synchronize()
    counts = K.kernel_counts()
    grads = {k: p.grad.detach().cpu().clone() for k, p in model.named_parameters()}
    if want_model:
        return pred.detach().cpu(), loss.item(), opt.last_norm.item(), grads, counts, model
    return pred.detach().cpu(), loss.item(), opt.last_norm.item(), grads, counts


def check_grads(grads, o_grads, bound, floor=None, factor=1.5, tag=""):
    """Every tensor's relative error below `bound`, or below factor x `floor[k]`;
    prints the five worst tensors (the per-tensor error map)."""
    errs = {k: rel(grads[k], og) for k, og in o_grads.items()}
    worst5 = sorted(((e, k) for k, e in errs.items()), reverse=True)[:5]
    print("%s worst gradients: %s" % (tag, "; ".join("%s %.3e" % (k, e) for e, k in worst5)))
    if floor:
        ratio5 = sorted(((e / max(floor[k], 1e-30), k) for k, e in errs.items()), reverse=True)[:5]
        print("%s worst ratios to the reference's own error: %s" % (
            tag, "; ".join("%s %.2f (%.3e / %.3e)" % (k, r, errs[k], floor[k]) for r, k in ratio5)))
    bad = {k: (e, floor[k] if floor else None) for k, e in errs.items()
           if e >= bound and (floor is None or e >= factor * floor[k])}
    assert not bad, bad
    return worst5[0]


def autocast_reference_grads(params, src, trg, dtype=torch.bfloat16):
    """The reference model's gradients under torch autocast (the oracle's
    functional model, on the GPU): the error the reference's own mixed precision
    carries (reference step: training_utils.py:64-70 with autocast); with
    dtype=float32, plain torch fp32 on the GPU."""
    p = {k: v.detach().clone().to(DEV).requires_grad_(True) for k, v in params.items()}
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype != torch.float32):
        pred = model_ref.seq2seq_forward(p, src.to(DEV), H)
    model_ref.loss_fn(pred.float(), trg.to(DEV)).backward()
    return {k: v.grad.detach().cpu() for k, v in p.items()}


def test_bf16_production_step_matches_oracle(problem):
    params, src, trg, o_loss, o_norm, o_pred, o_grads = problem
    pred, loss, norm, grads, c = run_step(params, src, trg, amp=True)
    # the kernels the 228M bench runs
    # every full-tile GEMM on the 4-wave persistent kernel (plain, bias, q|k|v+RoPE,
    # FFN1 ReLU-dropout, dReLU, the grouped weight gradients: one launch per decoder
    # layer, one per 4 encoder layers); the ring kernel keeps the f32 beta-1 dX
    # (residual accumulation) and the memory gradient
    n_grouped = L + L // 4
    assert c["gemm4"] >= 16 * L + n_grouped, c
    assert c["gemm4_tiles"] >= L * 256 + (L // 4) * 768, c
    assert c["gemm_group"] == 0, c
    assert c["attn_fwd"] == 3 * L and c["attn_bwd_fused"] == 3 * L, c
    assert c["attn_bwd_split"] == 0 and c["attn_fwd_generic"] == 0 and c["attn_bwd_generic"] == 0, c
    assert c["gemm_splitk_reduce"] <= 2, c  # only the 61-column head's weight gradient may split
    assert rel(pred, o_pred) < 3e-2
    mse = ((pred.double() - o_pred.double()) ** 2).mean().item()
    assert mse < 1e-3, mse
    assert abs(loss - o_loss.item()) < 2e-2 * abs(o_loss.item())
    assert abs(norm - o_norm.item()) < 2e-2 * o_norm.item()
    ac = autocast_reference_grads(params, src, trg)
    floor = {k: rel(ac[k], og) for k, og in o_grads.items()}
    worst = check_grads(grads, o_grads, 0.1, floor, tag="bf16 w3=1")
    print("bf16 production step: rel(pred) %.2e mse %.2e, worst grad %s" % (rel(pred, o_pred), mse, worst))


def test_fp32_production_step_matches_oracle(problem):
    params, src, trg, o_loss, o_norm, o_pred, o_grads = problem
    pred, loss, norm, grads, c = run_step(params, src, trg, amp=False)
    assert c["gemm_ring"] == 0 and c["gemm4"] == 0 and c["gemm128"] > 0, c  # fp32 parity mode: the 128 kernel
    assert c["attn_fwd"] == 3 * L and c["attn_bwd_split"] == 3 * L, c
    assert rel(pred, o_pred) < 1e-4
    assert ((pred.double() - o_pred.double()) ** 2).mean().item() < 1e-3
    assert abs(loss - o_loss.item()) < 1e-5 * abs(o_loss.item())
    assert abs(norm - o_norm.item()) < 1e-4 * o_norm.item()
    gg = autocast_reference_grads(params, src, trg, dtype=torch.float32)
    floor = {k: rel(gg[k], og) for k, og in o_grads.items()}
    worst = check_grads(grads, o_grads, 1e-4, floor, factor=2.0, tag="fp32 w3=1")
    print("fp32 production step: rel(pred) %.2e, worst grad %s" % (rel(pred, o_pred), worst))


def _ffn_relu_masks(model):
    """The ReLU pattern of our forward: FFN hidden > 0 per layer (the engine saves
    the post-ReLU hidden for the backward; dropout is 0 here)."""
    bb = model.engine().saved["bb"]
    out = {}
    for l, h in enumerate(bb.e_h):
        out["encoder.transformer_encoder.%d.ffn" % l] = (h > 0).cpu()
    for l, h in enumerate(bb.d_h):
        out["decoder.transformer_decoder.%d.ffn" % l] = (h > 0).cpu()
    return out


def _pinned_oracle_step(params, src, trg, masks, w3, monkeypatch):
    """The oracle's step with its ReLU derivative pinned to `masks` (the oracle's
    own forward otherwise): relu(z) = z * mask.  Returns the oracle's outputs and
    how many of its pre-activations fall on the other side of zero than ours."""
    flips = [0, 0]
    real_linear = model_ref.linear

    def ffn(p, name, x, dropout=0.0, training=False):
        z = real_linear(p, name + ".linear1", x)
        m = masks[name].view(z.shape)
        flips[0] += int(((z.detach() > 0) != m).sum())
        flips[1] += int((z.detach().abs() < 1e-6).sum())
        return real_linear(p, name + ".linear2", z * m.to(z.dtype))
    monkeypatch.setattr(model_ref, "ffn", ffn)
    oracle = model_ref.OracleTrainer(params, H, w3=w3)
    o_loss, o_norm, o_pred = oracle.step(src, trg)
    return o_loss, o_norm, o_pred, oracle.last_grads, flips


@pytest.mark.parametrize("w3", [0.0, 1.0])
def test_fp32_production_step_relu_pinned(problem, w3, monkeypatch):
    """fp32 kernels at the production shape to 1e-4, no floor.  Unpinned, the
    oracle's gradients differ from ours by ~1.2e-3, and the reference's own
    code run by torch in fp32 on the GPU differs from the CPU run by the same
    ~1.1e-3 with the loss's direction term off too (w3 = 0): at B*T = 16,384 a
    few dozen of the 2 x 4 x 67 M FFN pre-activations lie within f32 rounding of
    zero, and the side of zero each one lands on decides whether its ReLU passes
    a gradient (profiles/r3_production_parity.txt).  With the oracle's ReLU
    pattern pinned to our forward's, every gradient, the loss and the clip norm
    agree to 1e-4 relative, for the reference loss (w3 = 1) and without its
    direction term (w3 = 0)."""
    params, src, trg = problem[:3]
    pred, loss, norm, grads, c, model = run_step(params, src, trg, amp=False, w3=w3, want_model=True)
    masks = _ffn_relu_masks(model)
    del model
    o_loss, o_norm, o_pred, o_grads, flips = _pinned_oracle_step(params, src, trg, masks, w3, monkeypatch)
    print("fp32 w3=%g ReLU pinned: %d pre-activations on the other side of zero, %d within 1e-6 of it"
          % (w3, flips[0], flips[1]))
    worst = check_grads(grads, o_grads, 1e-4, tag="fp32 w3=%g ReLU pinned" % w3)
    # the clip norm against the float64 norm of the oracle's gradients: the oracle's
    # own f32 CPU norm (torch.stack of per-tensor norms) is itself ~1e-4 off it
    f64norm = lambda gs: sum(float(g.double().pow(2).sum()) for g in gs.values()) ** 0.5
    o_norm64 = f64norm(o_grads)
    print("norms: ours %.9g, float64 of the oracle's gradients %.9g (the oracle's f32 norm %.9g)"
          % (norm, o_norm64, o_norm.item()))
    assert rel(pred, o_pred) < 1e-4
    assert abs(loss - o_loss.item()) < 1e-5 * abs(o_loss.item())
    assert abs(norm - o_norm64) < 1e-5 * o_norm64
    print("fp32 production step, ReLU pinned, w3=%g: rel(pred) %.2e, norm rel %.2e, worst grad %s"
          % (w3, rel(pred, o_pred), abs(norm - o_norm64) / o_norm64, worst))


def test_bf16_production_step_no_direction_term(problem_w3_0):
    """bf16 step with w3 = 0: every gradient within 0.1 relative, no floor."""
    params, src, trg, o_loss, o_norm, o_pred, o_grads = problem_w3_0
    pred, loss, norm, grads, c = run_step(params, src, trg, amp=True, w3=0.0)
    assert rel(pred, o_pred) < 3e-2
    assert abs(loss - o_loss.item()) < 2e-2 * abs(o_loss.item())
    assert abs(norm - o_norm.item()) < 2e-2 * o_norm.item()
    worst = check_grads(grads, o_grads, 0.1, tag="bf16 w3=0")
    print("bf16 production step, w3=0: rel(pred) %.2e, worst grad %s" % (rel(pred, o_pred), worst))


def test_bf16_full_depth_step_matches_oracle():
    """The 228M configuration's full depth (L = 8 + 8, 235.5 M parameters) at
    B*T = 16,384 in bf16 with the reference loss: forward within 3e-2 relative and
    the metric's MSE gate, loss and clip norm within 2e-2, every gradient within
    0.1 relative or 2 x the reference's own bf16-autocast error on it.  At this
    depth the last decoder layer's self-attention q/k gradients (tiny,
    cancellation-dominated tensors) come out at 1.57-1.66 x that error, the head
    weight at 1.47 x, every other tensor below 1.5 x (two independent bf16
    roundings of the same computation; profiles/r3_production_parity.txt)."""
    Lf = 8
    params, src, trg, o_loss, o_norm, o_pred, o_grads = make_problem(Lf, 81, 1.0)
    pred, loss, norm, grads, c = run_step(params, src, trg, amp=True, n_layers=Lf)
    assert c["gemm_group"] == 0 and c["gemm4"] >= 16 * Lf + Lf + Lf // 4, c
    mse = ((pred.double() - o_pred.double()) ** 2).mean().item()
    assert rel(pred, o_pred) < 3e-2 and mse < 1e-3, (rel(pred, o_pred), mse)
    assert abs(loss - o_loss.item()) < 2e-2 * abs(o_loss.item())
    assert abs(norm - o_norm.item()) < 2e-2 * o_norm.item()
    ac = autocast_reference_grads(params, src, trg)
    floor = {k: rel(ac[k], og) for k, og in o_grads.items()}
    worst = check_grads(grads, o_grads, 0.1, floor, factor=2.0, tag="bf16 L=8")
    print("bf16 full-depth step: rel(pred) %.2e mse %.2e, loss rel %.2e, norm rel %.2e, worst grad %s"
          % (rel(pred, o_pred), mse, abs(loss - o_loss.item()) / abs(o_loss.item()),
             abs(norm - o_norm.item()) / o_norm.item(), worst))


def test_fp8_backward_production_step_vs_oracle(problem):
    """C5's fp8 step (e4m3 attention projections and encoder FFN linear1 forward,
    e4m3 FFN linear2 input gradients) at the production shape, held to the fp32
    ORACLE's gradients (not only to the bf16 step): e4m3's 3 mantissa bits put
    ~5 % relative error on a single GEMM, so every tensor is held to 0.35
    relative, or 2 x the bf16 step's own error on it, and the clip norm to 5 %."""
    params, src, trg, o_loss, o_norm, o_pred, o_grads = problem
    pred, loss, norm, grads, c = run_step(params, src, trg, amp=True, fp8=True)
    assert c["gemm_fp8"] >= 5 * L + 2 * L, c
    _, _, _, g16, _ = run_step(params, src, trg, amp=True)
    floor = {k: rel(g16[k], og) for k, og in o_grads.items()}
    worst = check_grads(grads, o_grads, 0.35, floor, factor=2.0, tag="fp8 fwd+bwd vs oracle")
    mse = ((pred.double() - o_pred.double()) ** 2).mean().item()
    print("fp8 step vs oracle: forward mse %.2e, loss %.4f vs %.4f, norm %.4f vs %.4f, worst grad %s"
          % (mse, loss, o_loss.item(), norm, o_norm.item(), worst))
    assert mse < 1e-3, mse
    assert abs(norm - o_norm.item()) < 0.05 * o_norm.item()
