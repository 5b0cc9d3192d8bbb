"""Feature-transform path (STNkd, the transform bmm, the
regulariser) on the HIP device vs the numpy oracle and the golden fixtures
g5 (forward) and g7 (run_training_pointnet_cls step with feature_transform=True)
captured from the reference.  Tolerance as in test_gpu_parity.py."""
import numpy as np
import pytest
import torch

from oracle import pointnet_np as onp
from golden_util import assert_grad_close, check_tensor, check_tensor_rel, load, rel_err

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from adversarial_learning_on_pointclouds_amd import ops
    from adversarial_learning_on_pointclouds_amd.pointnet import (PointNetCls, STNkd,
                                                                  feature_transform_regularizer)

DEV = "cuda"


def _t(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, dtype)


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("K,O,act", [(3, 64, 1), (64, 64, 1), (64, 128, 1), (128, 1024, 0),
                                     (64, 96, 0)])
def test_pw_fwd_vs_oracle(K, O, act):
    rng = np.random.default_rng(K + O)
    M = 200
    x = rng.normal(size=(M, K)).astype(np.float32)
    w = rng.normal(size=(O, K)).astype(np.float32) / np.sqrt(K)
    b = rng.normal(size=O).astype(np.float32)
    y = ops.pw_fwd(_t(x), _t(w), _t(b), act)
    ref = x @ w.T + b
    if act:
        ref = np.maximum(ref, 0)
    assert rel_err(_np(y), ref) < 1e-5


def test_transform_bmm_fwd_bwd():
    rng = np.random.default_rng(3)
    B, N, k = 3, 256, 64
    x = rng.normal(size=(B, N, k)).astype(np.float32)
    T = rng.normal(size=(B, k, k)).astype(np.float32) / 8
    dy = rng.normal(size=(B, N, k)).astype(np.float32)
    xt, Tt = _t(x).requires_grad_(True), _t(T).requires_grad_(True)
    y = ops.TransformFunction.apply(xt, Tt)
    y.backward(_t(dy))
    assert rel_err(_np(y), np.matmul(x, T)) < 1e-5
    assert rel_err(_np(xt.grad), np.matmul(dy, T.transpose(0, 2, 1))) < 1e-5
    assert rel_err(_np(Tt.grad), np.matmul(x.transpose(0, 2, 1), dy)) < 1e-5


@pytest.mark.parametrize("K,O", [(3, 64), (64, 64), (64, 128), (128, 128)])
def test_pw_bwd_vs_oracle(K, O):
    rng = np.random.default_rng(7 * K + O)
    M = 512
    x = rng.normal(size=(M, K)).astype(np.float32)
    w = rng.normal(size=(O, K, 1)).astype(np.float32) / np.sqrt(K)
    b = rng.normal(size=O).astype(np.float32)
    dy = rng.normal(size=(M, O)).astype(np.float32)
    xt = _t(x).requires_grad_(True)  # K = 3: the points' gradient (k_pw_bwd_data3)
    wt, bt = _t(w).requires_grad_(True), _t(b).requires_grad_(True)
    y = ops.PointwiseFunction.apply(xt, wt, bt, ops.ACT_RELU)
    y.backward(_t(dy))
    yr = np.maximum(x @ w[:, :, 0].T + b, 0)
    dW, db, dx = onp._layer_bwd(dy, x, yr, w[:, :, 0])
    assert rel_err(_np(wt.grad)[:, :, 0], dW) < 1e-5
    assert rel_err(_np(bt.grad), db) < 1e-5
    assert rel_err(_np(xt.grad), dx) < 1e-5


@pytest.mark.parametrize("relu", [False, True])
def test_conv_max_bwd_vs_oracle(relu):
    rng = np.random.default_rng(11 + relu)
    C, N, K, O = 4, 1024, 128, 1024
    x = np.maximum(rng.normal(size=(C, N, K)), 0).astype(np.float32)
    w = (rng.normal(size=(O, K)) / np.sqrt(K)).astype(np.float32)
    b = rng.normal(size=O).astype(np.float32)
    dg = rng.normal(size=(C, O)).astype(np.float32)
    xt, wt, bt = _t(x).requires_grad_(True), _t(w).requires_grad_(True), _t(b).requires_grad_(True)
    g = ops.ConvMaxFunction.apply(xt, wt, bt, relu)
    g.backward(_t(dg))
    gr, am = onp.conv_max_fwd(x, w, b, relu_before_max=relu)
    assert rel_err(_np(g), gr) < 1e-5
    dgm = dg * (gr > 0) if relu else dg
    dW, db, dX = onp.conv_max_bwd(dgm, am, x, w)
    assert rel_err(_np(wt.grad), dW) < 1e-5
    assert rel_err(_np(bt.grad), db) < 1e-5
    assert rel_err(_np(xt.grad), dX) < 1e-5


def test_regularizer_fwd_bwd():
    rng = np.random.default_rng(5)
    T = (np.eye(64)[None] + 0.1 * rng.normal(size=(6, 64, 64))).astype(np.float32)
    Tt = _t(T).requires_grad_(True)
    reg = feature_transform_regularizer(Tt)
    (0.5 * reg).backward()
    assert abs(reg.item() - onp.feature_transform_regularizer(T)) < 1e-5
    assert rel_err(_np(Tt.grad), 0.5 * onp.regularizer_bwd(T)) < 1e-5


def test_linear_identity_and_long_reduction():
    """STNkd fc3 (256 -> 64*64) + identity; its backward reduces over 4096."""
    rng = np.random.default_rng(9)
    x = rng.normal(size=(32, 256)).astype(np.float32)
    w = (rng.normal(size=(4096, 256)) / 16).astype(np.float32)
    b = rng.normal(size=4096).astype(np.float32)
    dy = rng.normal(size=(32, 4096)).astype(np.float32)
    xt, wt, bt = (_t(a).requires_grad_(True) for a in (x, w, b))
    y = ops.LinearFunction.apply(xt, wt, bt, ops.ACT_NONE, None, 0.0, 64)
    y.backward(_t(dy))
    ref = x @ w.T + b + np.eye(64, dtype=np.float32).reshape(1, -1)
    assert rel_err(_np(y), ref) < 1e-5
    assert rel_err(_np(xt.grad), dy @ w) < 1e-5
    assert rel_err(_np(wt.grad), dy.T @ x) < 1e-5


def _ft_model(seed):
    G = onp.make_params(onp.cls_ft_spec(40), seed=seed)
    m = PointNetCls(k=40, feature_transform=True)
    m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in G.items()})
    return m.to(DEV), G


def test_stnkd_module_vs_oracle():
    m, G = _ft_model(5)
    rng = np.random.default_rng(15)
    x = np.maximum(rng.normal(size=(2, 1024, 64)), 0).astype(np.float32)
    T = m.feat.fstn.forward_points(_t(x))
    assert rel_err(_np(T), onp.stn_forward(G, x, "feat.fstn.", 64)) < 1e-4
    # reference layout B x k x N
    T2 = m.feat.fstn(_t(x.transpose(0, 2, 1)))
    assert torch.equal(T, T2)


def test_cls_ft_forward_golden_g5():
    fx = load("g5_tnet.npz")
    m, _ = _ft_model(int(fx["g_seed"]))
    m.eval()
    pts = np.random.default_rng(int(fx["pts_seed"])).uniform(-1, 1, (2, 1024, 3)).astype(np.float32)
    with torch.no_grad():
        logits, glob, trans = m(_t(pts))
        reg = feature_transform_regularizer(trans)
    assert rel_err(_np(trans), fx["trans"]) < 1e-4
    assert rel_err(_np(glob)[:, :, 0], fx["gmax"]) < 1e-4
    assert rel_err(_np(logits), fx["logits"]) < 1e-4
    assert abs(reg.item() - float(fx["reg"])) < 1e-3


def test_cls_ft_step_golden_g7():
    """One run_training_pointnet_cls iteration (utils/trainer.py:254-268) with
    feature_transform=True: CE + 0.001 * regulariser, backward, Adam."""
    fx = load("g7_cls_ft_step.npz")
    m, G = _ft_model(int(fx["g_seed"]))
    m.train()
    m.dropout_masks = [_t(fx["mask"])]
    opt = torch.optim.Adam(m.parameters(), lr=1e-4, betas=(0.9, 0.999))
    opt.zero_grad()
    logits, _, trans = m(_t(fx["pts"]))
    l = torch.nn.functional.cross_entropy(logits, _t(fx["labels"], torch.int64))
    reg = feature_transform_regularizer(trans)
    loss = float(fx["lambda_cls"]) * l + float(fx["lambda_regu"]) * reg
    loss.backward()
    assert abs(l.item() - float(fx["loss_cls"])) < 1e-4
    assert abs(reg.item() - float(fx["reg"])) < 1e-3
    for name, p in m.named_parameters():
        check_tensor_rel(fx, "grad." + name, _np(p.grad), tol=1e-4)
    opt.step()
    for name, p in m.named_parameters():
        check_tensor(fx, "param." + name, _np(p), tol=1e-5)


def test_cls_ft_full_size_vs_oracle():
    """B=32, N=1024 feature-transform step against the oracle (gradients of all
    70 parameter tensors)."""
    m, G = _ft_model(17)
    rng = np.random.default_rng(171)
    B = 32
    pts = rng.uniform(-1, 1, (B, 1024, 3)).astype(np.float32)
    labels = rng.integers(0, 40, B)
    mask = (rng.random((B, 256)) >= 0.3).astype(np.float32)
    m.train()
    m.dropout_masks = [_t(mask)]
    logits, _, trans = m(_t(pts))
    l = torch.nn.functional.cross_entropy(logits, _t(labels, torch.int64))
    reg = feature_transform_regularizer(trans)
    (l + 0.001 * reg).backward()
    lr, rr, grads, aux = onp.cls_ft_step(G, pts, labels, mask, 1.0, 0.001)
    assert abs(l.item() - lr) < 1e-4 and abs(reg.item() - rr) < 1e-3
    for name, p in m.named_parameters():
        assert_grad_close(_np(p.grad), grads[name], name)


def _stn3d(seed):
    from adversarial_learning_on_pointclouds_amd.pointnet import STN3d
    S = onp.make_params(onp.stnkd_spec("", 3), seed=seed)
    m = STN3d()
    m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in S.items()})
    return m.to(DEV), S


def test_stn3d_golden_g12():
    """STN3d (models/pointnet.py:14-43, the 3x3 T-Net north_star names) on the
    reference layout B x 3 x N: forward and backward against the reference's own
    capture (g12): the transform, every parameter gradient per tensor and the
    input gradient."""
    fx = load("g12_stn3d.npz")
    m, _ = _stn3d(int(fx["s_seed"]))
    rng = np.random.default_rng(int(fx["data_seed"]))
    B, N = int(fx["B"]), int(fx["N"])
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    dT = rng.normal(0, 1, (B, 3, 3)).astype(np.float32)
    x = _t(pts.transpose(0, 2, 1)).requires_grad_(True)
    T = m(x)
    assert T.shape == (B, 3, 3)
    T.backward(_t(dT))
    assert rel_err(_np(T), fx["trans"]) < 1e-5
    for name, p in m.named_parameters():
        check_tensor_rel(fx, "grad." + name, _np(p.grad), tol=1e-4)
    check_tensor_rel(fx, "dx", _np(x.grad).transpose(0, 2, 1), tol=1e-4)


def test_stn3d_full_size_vs_oracle():
    """STN3d at B=32, N=1024 against the oracle's forward / backward: every
    gradient per tensor (default tolerance) and the input gradient."""
    m, S = _stn3d(33)
    rng = np.random.default_rng(331)
    B, N = 32, 1024
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    dT = rng.normal(0, 1, (B, 3, 3)).astype(np.float32)
    x = _t(pts.transpose(0, 2, 1)).requires_grad_(True)
    T = m(x)
    T.backward(_t(dT))
    Tr, cache = onp.stn_forward_train(S, pts, "", 3)
    grads, dx = onp.stn_backward(S, cache, dT, "")
    assert rel_err(_np(T), Tr) < 1e-5
    for name, p in m.named_parameters():
        assert_grad_close(_np(p.grad), grads[name], name)
    assert_grad_close(_np(x.grad).transpose(0, 2, 1), dx, "dx")


@pytest.mark.parametrize("ft", [False, True])
def test_pointnetfeat_dense_vs_oracle(ft):
    """PointNetfeat(global_feat=False) (models/pointnet.py:133-137): the global
    feature repeated over the points, then conv2's point features (after the
    feature transform when on): B x 1088 x N, and its backward through both."""
    from adversarial_learning_on_pointclouds_amd.pointnet import PointNetfeat
    spec = onp.cls_ft_spec(40) if ft else onp.cls_spec(40)
    G = onp.make_params(spec, seed=21)
    f = PointNetfeat(global_feat=False, feature_transform=ft)
    f.load_state_dict({k[len("feat."):]: torch.from_numpy(v.copy()) for k, v in G.items()
                       if k.startswith("feat.")})
    f = f.to(DEV)
    rng = np.random.default_rng(22)
    B, N = 2, 512  # the feature transform takes N % 256 == 0 (its dT per-cloud row groups)
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    x = _t(pts.transpose(0, 2, 1)).requires_grad_(True)
    out, trans = f(x)
    assert out.shape == (B, 1088, N) and (trans is not None) == ft
    x1, x2, _ = onp.point_mlp_fwd(pts, G)
    if ft:
        T = onp.stn_forward(G, x2, "feat.fstn.", 64)
        x2 = np.matmul(x2, T)
        x3 = np.maximum(x2 @ onp._w(G, "feat.conv3.weight").T + G["feat.conv3.bias"], 0)
    else:
        _, _, x3 = onp.point_mlp_fwd(pts, G)
    gmax, _ = onp.conv_max_fwd(x3, onp._w(G, "feat.conv4.weight"), G["feat.conv4.bias"])
    ref = np.concatenate([np.repeat(gmax[:, :, None], N, 2), x2.transpose(0, 2, 1)], 1)
    assert rel_err(_np(out), ref) < 1e-4
    # backward: a cotangent on the point features only reaches conv1 / conv2
    # (and the transform); one on the global part goes through the max-pool
    dy = rng.normal(size=(B, 1088, N)).astype(np.float32)
    out.backward(_t(dy))
    assert torch.isfinite(x.grad).all() and float(x.grad.abs().sum()) > 0
    assert f.conv1.weight.grad is not None and f.conv4.weight.grad is not None
    if not ft:  # dW4 from the pooled gradient: sum over points of dy's global rows
        dg = dy[:, :1024, :].sum(2)
        _, am = onp.conv_max_fwd(x3, onp._w(G, "feat.conv4.weight"), G["feat.conv4.bias"])
        dw4 = np.einsum("bo,bok->ok", dg, x3[np.arange(B)[:, None], am])
        assert rel_err(_np(f.conv4.weight.grad)[:, :, 0], dw4) < 1e-4


@pytest.mark.parametrize("relu,N", [(False, 333), (True, 333), (True, 64)])
def test_conv_max_1024_ragged_vs_oracle(relu, N):
    """The 1024-channel conv + max (feature conv4 / T-Net conv3) runs on
    k_conv4_max: ragged point counts, the ReLU-before-max fix-up (an
    all-negative channel pools 0 at point 0, as torch.max over the zeros), and
    the argmax the backward routes through."""
    rng = np.random.default_rng(90 + N + relu)
    C, K, O = 3, 128, 1024
    x = np.maximum(rng.normal(size=(C, N, K)), 0).astype(np.float32)
    w = (rng.normal(size=(O, K)) / np.sqrt(K)).astype(np.float32)
    b = (rng.normal(size=O) - (2.0 if relu else 0.0)).astype(np.float32)  # many all-negative channels
    gmax, gidx = ops.conv_max_fwd(_t(x), _t(w), _t(b), relu)
    gr, am = onp.conv_max_fwd(x, w, b, relu_before_max=relu)
    assert rel_err(_np(gmax), gr) < 1e-5
    gi = _np(gidx)
    # exact argmax except near-ties of the f32 values (different summation orders)
    y = np.einsum("cnk,ok->con", x.astype(np.float64), w.astype(np.float64)) + b[None, :, None]
    if relu:
        y = np.maximum(y, 0)
    top = y.max(2)
    picked = np.take_along_axis(y, gi[:, :, None].astype(np.int64), 2)[:, :, 0]
    ok = (gi == am) | (np.abs(top - picked) <= 1e-5 * (np.abs(top) + 1e-6))
    assert ok.all()
    if relu:
        zero = gr == 0
        assert zero.any() and (gi[zero] == 0).all() and (_np(gmax)[zero] == 0).all()
