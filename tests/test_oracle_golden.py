"""Pin the numpy oracle against golden vectors captured from the reference.

CPU only.  The fixtures come from tests/golden/make_golden.py, which ran the
reference's own modules (models/pointnet.py, models/discriminator.py,
utils/trainer.py:run_training) on the same seeded inputs.
"""
import numpy as np
import pytest

from oracle import pointnet_np as onp
from golden_util import load, rel_err, check_tensor, check_tensor_rel


def _pts(seed, B, N):
    return np.random.default_rng(seed).uniform(-1, 1, (B, N, 3)).astype(np.float32)


def test_g1_cls_forward():
    fx = load("g1_cls_fwd.npz")
    G = onp.make_params(onp.cls_spec(40), seed=int(fx["g_seed"]))
    pts = _pts(int(fx["pts_seed"]), int(fx["B"]), int(fx["N"]))
    logits, gmax, cache = onp.cls_forward(G, pts, None)
    assert rel_err(logits, fx["logits"]) < 1e-4
    assert rel_err(gmax, fx["gmax"]) < 1e-4
    assert (cache["am"] == fx["argmax"]).mean() > 0.999


def test_g2_cls_backward():
    fx = load("g2_cls_bwd.npz")
    G = onp.make_params(onp.cls_spec(40), seed=int(fx["g_seed"]))
    pts = _pts(int(fx["pts_seed"]), 4, 1024)
    logits, _, cache = onp.cls_forward(G, pts, fx["mask"])
    loss, dlog = onp.cross_entropy(logits, fx["labels"])
    assert abs(loss - float(fx["loss"])) < 1e-5
    grads = onp.cls_backward(G, cache, dlog)
    for k in G:
        check_tensor_rel(fx, "grad." + k, grads[k], tol=1e-4)


def _adv_inputs(fx):
    rng = np.random.default_rng(int(fx["data_seed"]))
    B, N, iters = int(fx["B"]), int(fx["N"]), int(fx["iters"])
    steps = []
    for _ in range(iters):
        pg = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
        lab = rng.integers(0, 40, B)
        pn = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
        m1 = (rng.random((B, 256)) >= 0.3).astype(np.float32)
        m2 = (rng.random((B, 256)) >= 0.3).astype(np.float32)
        y1 = rng.uniform(0.7, 1.05, (B, 1)).astype(np.float32)
        y2 = rng.uniform(0.0, 0.305, (B, 1)).astype(np.float32)
        steps.append((pg, lab, pn, m1, m2, y1, y2))
    return steps


@pytest.mark.parametrize("name", ["g3_adv_step1.npz", "g3_adv_step3.npz", "g3_adv_step1_b32.npz"])
def test_g3_adv_step(name):
    fx = load(name)
    G = onp.make_params(onp.cls_spec(40), seed=int(fx["g_seed"]))
    D = onp.make_params(onp.disc_spec(40, 1), seed=int(fx["d_seed"]), init="xavier")
    oG, oD = onp.Adam(G), onp.Adam(D)
    for i, (pg, lab, pn, m1, m2, y1, y2) in enumerate(_adv_inputs(fx)):
        losses, gG, gD, _ = onp.adv_step(G, D, oG, oD, pg, lab, pn, m1, m2, y1, y2)
        assert abs(losses["loss_cls"] - fx["loss_cls"][i]) < 1e-4
        assert abs(losses["loss_adv"] - fx["loss_adv"][i]) < 1e-4
        assert abs(losses["loss_D_gt"] - fx["loss_D_gt"][i]) < 1e-4
        assert abs(losses["loss_D_nogt"] - fx["loss_D_nogt"][i]) < 1e-4
        if int(fx["iters"]) == 1:
            for k in G:
                check_tensor_rel(fx, "gradG." + k, gG[k], tol=1e-4)
            for k in D:
                check_tensor_rel(fx, "gradD." + k, gD[k], tol=1e-4)
    for k in G:
        check_tensor(fx, "paramG." + k, G[k], tol=1e-5)
    for k in D:
        check_tensor(fx, "paramD." + k, D[k], tol=1e-5)


def test_g9_semi_step():
    """run_training_semi (utils/trainer.py:611-847), 3 iterations, the
    pseudo-label term on from i_iter 2 with half the no-GT clouds kept."""
    fx = load("g9_semi_step3.npz")
    G = onp.make_params(onp.cls_spec(40), seed=int(fx["g_seed"]))
    D = onp.make_params(onp.disc_spec(40, 1), seed=int(fx["d_seed"]), init="xavier")
    oG, oD = onp.Adam(G), onp.Adam(D)
    semi_start, th = int(fx["semi_start"]), float(fx["semi_th"])
    semi_losses = []
    for i, (pg, lab, pn, m1, m2, y1, y2) in enumerate(_adv_inputs(fx)):
        on = semi_start > 0 and i > semi_start
        losses, _, _, _ = onp.adv_step(G, D, oG, oD, pg, lab, pn, m1, m2, y1, y2, semi=on,
                                       semi_th=th, lambda_semi=float(fx["lambda_semi"]))
        assert abs(losses["loss_cls"] - fx["loss_cls"][i]) < 1e-4
        assert abs(losses["loss_adv"] - fx["loss_adv"][i]) < 1e-4
        assert abs(losses["loss_D_gt"] - fx["loss_D_gt"][i]) < 1e-4
        assert abs(losses["loss_D_nogt"] - fx["loss_D_nogt"][i]) < 1e-4
        if on:
            assert losses["semi_ratio"] == float(fx["semi_ratio"])
            semi_losses.append(losses["loss_semi"])
    assert np.allclose(semi_losses, fx["loss_semi"], atol=1e-4)
    for k in G:
        check_tensor(fx, "paramG." + k, G[k], tol=1e-5)
    for k in D:
        check_tensor(fx, "paramD." + k, D[k], tol=1e-5)


def test_g4_disc():
    fx = load("g4_disc.npz")
    D = onp.make_params(onp.disc_spec(40, 1), seed=int(fx["d_seed"]), init="xavier")
    out, acts = onp.disc_forward(D, fx["x"])
    assert rel_err(out, fx["out"]) < 1e-5
    g, dx = onp.disc_backward(D, acts, fx["dout"])
    assert rel_err(dx, fx["dx"]) < 1e-5
    for k in D:
        check_tensor_rel(fx, "grad." + k, g[k], tol=1e-5)


def test_g5_tnet():
    fx = load("g5_tnet.npz")
    G = onp.make_params(onp.cls_ft_spec(40), seed=int(fx["g_seed"]))
    pts = _pts(int(fx["pts_seed"]), 2, 1024)
    logits, gmax, trans = onp.cls_ft_forward(G, pts)
    assert rel_err(trans, fx["trans"]) < 1e-4
    assert rel_err(gmax, fx["gmax"]) < 1e-4
    assert rel_err(logits, fx["logits"]) < 1e-4
    assert abs(onp.feature_transform_regularizer(trans) - float(fx["reg"])) < 1e-3


def test_g6_seg():
    fx = load("g6_seg_fwd.npz")
    S = onp.make_params(onp.seg_spec(50), seed=int(fx["s_seed"]))
    pts = _pts(int(fx["pts_seed"]), 2, 2048)
    out, g = onp.seg_forward(S, pts, fx["cls"])
    assert rel_err(g[:, :, 0], fx["gmax"]) < 1e-4
    check_tensor(fx, "out", out, tol=1e-4)


def test_g7_cls_ft_step():
    """run_training_pointnet_cls with feature_transform=True (T-Net path, SURVEY
    row a7): CE + 0.001 * regularizer, gradients of every parameter and the
    parameters after the Adam step."""
    fx = load("g7_cls_ft_step.npz")
    G = onp.make_params(onp.cls_ft_spec(40), seed=int(fx["g_seed"]))
    l, reg, grads, _ = onp.cls_ft_step(G, fx["pts"], fx["labels"], fx["mask"],
                                       float(fx["lambda_cls"]), float(fx["lambda_regu"]))
    assert abs(l - float(fx["loss_cls"])) < 1e-4
    assert abs(reg - float(fx["reg"])) < 1e-3
    for name, g in grads.items():
        check_tensor_rel(fx, "grad." + name, g, tol=1e-4)
    opt = onp.Adam(G)
    opt.step(grads)
    for name, v in G.items():
        check_tensor(fx, "param." + name, v, tol=1e-5)


def test_g8_seg_step():
    """run_training_pointnet_seg (BASELINE configs[3]):
    PointNetSeg forward, per-point CrossEntropyLoss, gradients of every
    parameter (strict relative form) and the parameters after one Adam step."""
    fx = load("g8_seg_step.npz")
    S = onp.make_params(onp.seg_spec(50), seed=int(fx["s_seed"]))
    B, N = fx["seg"].shape
    pts = np.random.default_rng(int(fx["pts_seed"])).uniform(-1, 1, (B, N, 3)).astype(np.float32)
    loss, grads, logits, gmax, _ = onp.seg_step(S, pts, fx["cls"], fx["seg"])
    assert abs(loss - float(fx["loss"])) < 1e-5 * max(1.0, abs(float(fx["loss"])))
    check_tensor_rel(fx, "gmax", gmax, tol=1e-5)
    check_tensor_rel(fx, "logits", logits.transpose(0, 2, 1), tol=1e-5)
    for name, g in grads.items():
        check_tensor_rel(fx, "grad." + name, g, tol=1e-4)
    opt = onp.Adam(S)
    opt.step(grads)
    for name, v in S.items():
        check_tensor(fx, "param." + name, v, tol=1e-5)


def test_g11_cls_full_size():
    """configs[1] at full size (B=32, N=1024): the reference's loss, logits,
    global feature and every gradient."""
    fx = load("g11_cls_b32.npz")
    G = onp.make_params(onp.cls_spec(40), seed=int(fx["g_seed"]))
    rng = np.random.default_rng(int(fx["data_seed"]))
    B = int(fx["B"])
    pts = rng.uniform(-1, 1, (B, int(fx["N"]), 3)).astype(np.float32)
    lab = rng.integers(0, 40, B)
    mask = (rng.random((B, 256)) >= 0.3).astype(np.float32)
    logits, gmax, cache = onp.cls_forward(G, pts, mask)
    assert rel_err(logits, fx["logits"]) < 1e-5
    assert rel_err(gmax, fx["gmax"]) < 1e-5
    loss, dlog = onp.cross_entropy(logits, lab)
    assert abs(loss - float(fx["loss"])) < 1e-5
    grads = onp.cls_backward(G, cache, dlog)
    for k in G:
        check_tensor_rel(fx, "grad." + k, grads[k], tol=1e-4)


def test_bf16_mode_oracle_close_to_reference_g11():
    """The oracle's bf16 mode (conv3 / conv4 on bf16-rounded operands: the
    build's configs[1] variant, not a reference behaviour) stays close to the
    reference's fp32 outputs (g11): logits within 2e-2 of their scale, loss
    within 1e-2."""
    fx = load("g11_cls_b32.npz")
    G = onp.make_params(onp.cls_spec(40), seed=int(fx["g_seed"]))
    rng = np.random.default_rng(int(fx["data_seed"]))
    B = int(fx["B"])
    pts = rng.uniform(-1, 1, (B, int(fx["N"]), 3)).astype(np.float32)
    lab = rng.integers(0, 40, B)
    mask = (rng.random((B, 256)) >= 0.3).astype(np.float32)
    logits, gmax, _ = onp.cls_forward(G, pts, mask, precision="bf16")
    scale = np.abs(fx["logits"]).max()
    assert np.abs(logits - fx["logits"]).max() <= 2e-2 * scale
    loss, _ = onp.cross_entropy(logits, lab)
    assert abs(loss - float(fx["loss"])) < 1e-2
    assert not np.array_equal(logits, fx["logits"])  # the mode does change the arithmetic


def test_g12_stn3d():
    """STN3d (models/pointnet.py:14-43, the 3x3 T-Net of north_star) forward and
    backward against the reference's capture: the transform, every parameter
    gradient (strict per-tensor form) and the input gradient."""
    fx = load("g12_stn3d.npz")
    S = onp.make_params(onp.stnkd_spec("", 3), seed=int(fx["s_seed"]))
    rng = np.random.default_rng(int(fx["data_seed"]))
    B, N = int(fx["B"]), int(fx["N"])
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    dT = rng.normal(0, 1, (B, 3, 3)).astype(np.float32)
    T, cache = onp.stn_forward_train(S, pts, "", 3)
    assert rel_err(T, fx["trans"]) < 1e-5
    assert rel_err(onp.stn_forward(S, pts, "", 3), fx["trans"]) < 1e-5
    grads, dx = onp.stn_backward(S, cache, dT, "")
    for k in S:
        check_tensor_rel(fx, "grad." + k, grads[k], tol=1e-4)
    check_tensor_rel(fx, "dx", dx, tol=1e-4)


def test_adam_update_check_is_sensitive():
    """The update check of the fused-Adam GPU tests (golden_util.adam_update_err):
    an Adam at the right lr passes with a gradient perturbed at the GPU tests'
    tolerance (1e-3 of each tensor's max), one at half the lr fails every
    tensor, and so does one with eps inside the square root."""
    from golden_util import adam_update_err
    fx = load("g3_adv_step1.npz")
    G = onp.make_params(onp.cls_spec(40), seed=int(fx["g_seed"]))
    D = onp.make_params(onp.disc_spec(40, 1), seed=int(fx["d_seed"]), init="xavier")
    pg, lab, pn, m1, m2, y1, y2 = _adv_inputs(fx)[0]
    _, gG, _, _ = onp.adv_step(G, D, None, None, pg, lab, pn, m1, m2, y1, y2, apply_adam=False)
    old = {k: v.copy() for k, v in G.items()}
    rng = np.random.default_rng(0)

    def run(lr=1e-4, eps=1e-8, noise=0.0):
        P = {k: v.copy() for k, v in old.items()}
        g = {k: (v + noise * np.abs(v).max() * rng.uniform(-1, 1, v.shape)).astype(np.float32)
             for k, v in gG.items()}
        onp.Adam(P, lr=lr, eps=eps).step(g)
        return P

    ref = run()
    ok, half = run(noise=1e-3), run(lr=0.5e-4)
    # eps misplaced: sqrt(v + eps) instead of sqrt(v) + eps (v = g^2 after step 1)
    bad_eps = {k: (old[k] - np.float32(1e-4) * gG[k] / (np.sqrt(gG[k].astype(np.float64) ** 2 + 1e-8)
                                                       )).astype(np.float32) for k in old}
    for k in G:
        e, n = adam_update_err(ok[k], old[k], ref[k], old[k], gG[k])
        assert n > 0 and e < 1e-3, (k, e)
        assert adam_update_err(half[k], old[k], ref[k], old[k], gG[k])[0] > 0.4, k
        # eps moves the update only where |g| is within a few decades of it: the
        # feature layers' small gradients
        if k.startswith("feat.") and k.endswith("weight"):
            assert adam_update_err(bad_eps[k], old[k], ref[k], old[k], gG[k])[0] > 2e-3, k


def test_g13_adv_ft_grads_first_iteration():
    """oracle.adv_ft_grads (run_training's body with a feature-transform
    generator, utils/trainer.py:467-556) against the reference's own first
    iteration of g13 ft_pool0 (same parameters, batches, dropout masks and soft
    labels): losses and every G / D gradient.  It is the checker of the GPU's
    same-activation test at iteration 3 (test_gpu_g13.py)."""
    fx = load("g13_adv_off_fused.npz")
    G = onp.make_params(onp.cls_ft_spec(40), seed=int(fx["g_seed"]))
    D = onp.make_params(onp.disc_spec(40, 1), seed=int(fx["d_seed"]), init="xavier")
    m, y = fx["masks"][0], fx["soft"][0]
    losses, gG, gD, _ = onp.adv_ft_grads(G, D, fx["pts_gt"][0], fx["labels"][0], fx["pts_nogt"][0],
                                         m[0], m[1], y[0][:, None], y[1][:, None],
                                         float(fx["lambda_cls"]), float(fx["lambda_adv"]))
    for k in ("loss_cls", "loss_adv", "loss_D_gt", "loss_D_nogt"):
        assert abs(losses[k] - float(fx[f"ft_pool0.{k}"][0])) < 1e-5, k
    for tag, grads in (("G", gG), ("D", gD)):
        for name, g in grads.items():
            check_tensor_rel(fx, f"ft_pool0.grad1{tag}.{name}", g, tol=1e-4)
