"""Pin the CPU oracle against fixtures generated from the reference (CPU only)."""
import numpy as np
import pytest
import torch

from oracle import data_ref, model_ref
from tests.golden.make_goldens_helpers import summary, synth_audio


def test_loss_matches_reference(golden):
    g = golden("loss.npz")
    for case in ("random", "zero_target", "zero_pred_diff", "small"):
        p = torch.tensor(g[case + "_pred"], requires_grad=True)
        t = torch.tensor(g[case + "_trg"])
        loss = model_ref.loss_fn(p, t)
        loss.backward()
        assert abs(loss.item() - float(g[case + "_loss"])) <= 1e-6 * max(1.0, abs(float(g[case + "_loss"])))
        np.testing.assert_allclose(p.grad.numpy(), g[case + "_grad"], rtol=1e-5, atol=1e-6 * np.abs(g[case + "_grad"]).max())


def test_rope_matches_reference(golden):
    g = golden("rope.npz")
    out = model_ref.global_pe(torch.tensor(g["x"]))
    np.testing.assert_array_equal(out.numpy(), g["global_out"])
    np.testing.assert_array_equal(model_ref.head_rope(torch.tensor(g["q"])).numpy(), g["q_out"])
    np.testing.assert_array_equal(model_ref.head_rope(torch.tensor(g["k"])).numpy(), g["k_out"])


@pytest.mark.parametrize("tag", ["tiny", "mid"])
def test_model_step_matches_reference(golden, tag):
    g = golden("model_%s.npz" % tag)
    D, H, L, seed = int(g["D"]), int(g["H"]), int(g["L"]), int(g["seed"])
    params = model_ref.seeded_params(model_ref.param_shapes(256, D, L, 61), seed)
    tr = model_ref.OracleTrainer(params, H)
    keys = list(params.keys())
    for s in range(int(g["steps"])):
        loss, total, pred = tr.step(torch.tensor(g["src%d" % s]), torch.tensor(g["trg%d" % s]))
        np.testing.assert_allclose(pred.numpy(), g["pred%d" % s], rtol=1e-4, atol=1e-4)
        assert abs(loss.item() - float(g["loss%d" % s])) < 1e-5 * abs(float(g["loss%d" % s]))
        assert abs(total.item() - float(g["gnorm%d" % s])) < 1e-4 * float(g["gnorm%d" % s])
        got = np.stack([summary(tr.p[k].detach().numpy()) for k in keys])
        np.testing.assert_allclose(got, g["params%d" % s], rtol=1e-5, atol=1e-6)


def test_adam_l2_matches_torch():
    torch.manual_seed(0)
    ps = [torch.randn(7, 5), torch.randn(11)]
    ref = [p.clone().requires_grad_(True) for p in ps]
    opt = torch.optim.Adam(ref, lr=1e-2, weight_decay=1e-2)
    mine = [p.clone() for p in ps]
    m = [torch.zeros_like(p) for p in ps]
    v = [torch.zeros_like(p) for p in ps]
    for step in range(1, 6):
        grads = [torch.randn_like(p) for p in ps]
        for r, gr in zip(ref, grads):
            r.grad = gr.clone()
        opt.step()
        model_ref.adam_l2_step(mine, [gr.clone() for gr in grads], m, v, step, 1e-2, weight_decay=1e-2)
        for a, b in zip(mine, ref):
            torch.testing.assert_close(a, b.detach(), rtol=0, atol=0)


def test_clip_matches_torch():
    torch.manual_seed(1)
    gs = [torch.randn(13, 3) * 3, torch.randn(40)]
    ps = [torch.zeros_like(g, requires_grad=True) for g in gs]
    for p, g in zip(ps, gs):
        p.grad = g.clone()
    tot = torch.nn.utils.clip_grad_norm_(ps, 2.0)
    mine = [g.clone() for g in gs]
    tot2 = model_ref.clip_grad_norm(mine, 2.0)
    assert abs(tot.item() - tot2.item()) < 1e-6 * tot.item()
    for a, p in zip(mine, ps):
        torch.testing.assert_close(a, p.grad, rtol=1e-6, atol=1e-7)


def test_lr_lambda_matches_reference(golden):
    g = golden("lr.npz")
    for warm in (0, 3):
        got = [model_ref.lr_lambda(e, warm, 50) for e in range(52)]
        np.testing.assert_allclose(got, g["warm%d" % warm], rtol=1e-12)


def test_full_width_layers_match_reference(golden):
    g = golden("layers_full.npz")
    rng = np.random.default_rng(7)
    x = torch.tensor(rng.standard_normal((1, 128, 1024)).astype(np.float32))
    mem = torch.tensor(rng.standard_normal((1, 128, 1024)).astype(np.float32))
    from tests.golden.make_goldens_helpers import full_layer_params
    pe, pd_ = full_layer_params()
    with torch.no_grad():
        ye = model_ref.encoder_layer(pe, "e", x, 16)
        yd = model_ref.decoder_layer(pd_, "d", x, mem, 16)
    np.testing.assert_allclose(ye.numpy()[0, ::17], g["enc_rows"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(yd.numpy()[0, ::17], g["dec_rows"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(summary(ye.numpy())[:2], g["enc_out"][:2], rtol=1e-4)


# ---------------------------------------------------------------------------
# data path: bit-exact
# ---------------------------------------------------------------------------
def test_window_plan_matches_reference(golden):
    g = golden("data_windows.npz")
    for n in (128, 256, 300, 1848, 129):
        starts = np.array([s for s, _ in data_ref.window_plan(n, n, 128)])
        np.testing.assert_array_equal(starts, g["starts_%d" % n])
    assert int(g["short_raises"]) == 1
    with pytest.raises(ValueError):
        data_ref.window_plan(100, 100, 128)


def test_augment_matches_reference_bitexact(golden):
    g = golden("data_augment.npz")
    for tag in "abcde":
        fast, slow = (bool(v) for v in g[tag + "_flags"])
        a, f = data_ref.augment(g[tag + "_audio_in"], g[tag + "_facial_in"], fast, slow)
        np.testing.assert_array_equal(a, g[tag + "_audio_out"])
        np.testing.assert_array_equal(f, g[tag + "_facial_out"])
    np.testing.assert_array_equal(data_ref.interpolate_slower(g["interp_in"]), g["interp_out"])
    np.testing.assert_array_equal(data_ref.smooth_facial_data(g["interp_in"]), g["smooth_out"])
    seqs = [g["blend_in0"], g["blend_in1"], g["blend_in2"]]
    np.testing.assert_array_equal(data_ref.stack_with_blend(seqs, 30), g["blend_out"])


def test_autocorr_matches_reference(golden):
    g = golden("features_autocorr.npz")
    for seconds, seed in ((1.0, 3), (0.73, 4)):
        y = synth_audio(seconds, seed)
        got = data_ref.reduce_features(data_ref.autocorr_features_120(y)).T
        np.testing.assert_allclose(got, g["ac_%d" % seed], rtol=1e-9, atol=1e-12)
    y = synth_audio(0.5, 5)
    y[:3000] = 0
    y[-3000:] = 0
    got = data_ref.reduce_features(data_ref.autocorr_features_120(y)).T
    np.testing.assert_allclose(got, g["ac_silent_edges"], rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(data_ref.reduce_features(g["reduce_in"]), g["reduce_out"])
    np.testing.assert_array_equal(data_ref.reduce_features(g["reduce_in_even"]), g["reduce_out_even"])
    np.testing.assert_allclose(data_ref.cmvn(g["reduce_in"]), g["cmvn_out"], rtol=1e-14)


def test_mfcc_restatement_properties():
    """Parity UNPINNED (no librosa here): check the restatement's own invariants."""
    y = synth_audio(1.0, 3)
    m = data_ref.mfcc_120(y, 88200)
    assert m.shape == (23, 1 + len(y) // 735)
    basis = data_ref.mel_basis(88200, 1470)
    assert basis.shape == (128, 736) and (basis.max(axis=1) > 0).all()
    c = data_ref.dct_ortho_matrix(128, 128)
    np.testing.assert_allclose(c @ c.T, np.eye(128), atol=1e-12)
    feats = data_ref.extract_features(y)
    assert feats.shape == ((1 + len(y) // 735 + 1) // 2, 256)
    assert data_ref.extract_features(y[:1470 + 7 * 735]) is None
