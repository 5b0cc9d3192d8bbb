"""Segmentation path (BASELINE configs[3]): the dense point-wise
GEMM engine (csrc/gemm.hip) through its C ABI, and PointNetSeg on top of it,
against float64 torch references, the numpy oracle and the reference goldens
g6 (forward) / g8 (training step).  Runs on an MI355X only.

Tolerances.  precision="fp32" (the default, the reference's dtype): every GEMM
takes six MFMA products of hi/mid/lo bf16 splits (f32-level); conv6's pooled
values are exact f32 re-evaluations.  The forward outputs (logits, x_global)
are held to the north_star's 1e-3 (they agree to ~1e-6); the backward to 1e-4
elementwise against the oracle's backward evaluated on this forward's own
activations and ReLU masks, and end to end in relative L2 within 2e-3 (two f32
implementations of a ReLU net route a whole gradient element differently where
a pre-activation lies within rounding of 0).  conv6's argmax must be the f64
argmax of the kernel's own conv5 activations except at proven near-ties
(_conv6_argmax_ok).  precision="bf16x3" (a labelled speed option): the
forward and data-gradient GEMMs take three products of hi/lo splits, bounded
by 2e-5 * (|A| |B|^T) elementwise; end to end 1e-2."""
import ctypes
import os

import numpy as np
import pytest
import torch

from oracle import pointnet_np as onp
from golden_util import check_tensor_l2, check_tensor_rel, load

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from adversarial_learning_on_pointclouds_amd import _lib
    from adversarial_learning_on_pointclouds_amd._lib import check, stream_ptr
    from adversarial_learning_on_pointclouds_amd.seg import (PointNetSeg, seg_backward,
                                                             seg_cross_entropy, seg_forward)

DEV = "cuda"


def _p(t, off=0):
    return ctypes.c_void_p(t.data_ptr() + 4 * off)


def _t(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, dtype)


def _bound(A, B):
    return 2e-5 * (np.abs(A) @ np.abs(B).T) + 1e-30


@pytest.mark.parametrize("M,N,K", [(300, 50, 70), (128, 128, 32), (1000, 256, 960), (7, 2048, 3)])
def test_gemm_forward_vs_fp64(M, N, K):
    lib = _lib.load()
    rng = np.random.default_rng(M + N + K)
    A = rng.standard_normal((M, K)).astype(np.float32)
    W = rng.standard_normal((N, K)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    br = rng.standard_normal((2, N)).astype(np.float32)
    C = torch.empty(M, N, device=DEV)
    rpg = (M + 1) // 2
    tA, tW, tb, tbr = _t(A), _t(W), _t(b), _t(br)  # alive across the launch
    check(lib.pcadv_gemm(_p(tA), K, 0, _p(tW), K, 0, _p(C), N, M, N, K, _p(tb), _p(tbr),
                         rpg, 1, 0, None, 0, 0, None, None, 0, stream_ptr()), "gemm")
    ref = A.astype(np.float64) @ W.astype(np.float64).T + b + br[np.arange(M) // rpg]
    ref = np.maximum(ref, 0)
    assert (np.abs(C.cpu().numpy() - ref) <= _bound(A, W) + 1e-6).all()


def test_gemm_data_grad_masked_accumulate():
    """dX = [Y > 0] (dX + dZ W) with a strided, offset output and a mask stored
    like it (the seg backward's form: the producer applies the next relu')."""
    lib = _lib.load()
    rng = np.random.default_rng(3)
    M, O, K = 517, 128, 64
    dZ = rng.standard_normal((M, O)).astype(np.float32)
    Y = rng.standard_normal((M, 200)).astype(np.float32)
    W = rng.standard_normal((O, K)).astype(np.float32)
    base = rng.standard_normal((M, 200)).astype(np.float32)
    out = _t(base)
    tdZ, tY, tW = _t(dZ), _t(Y), _t(W)
    check(lib.pcadv_gemm(_p(tdZ), O, 0, _p(tW), K, 1, _p(out, 64), 200, M, K, O, None, None, 0, 0,
                         1, _p(tY, 64), 200, 1, None, None, 0, stream_ptr()), "gemm")
    ref = base.astype(np.float64).copy()
    ref[:, 64:128] = (ref[:, 64:128] + dZ.astype(np.float64) @ W.astype(np.float64)) * (Y[:, 64:128] > 0)
    got = out.cpu().numpy()
    # six-product (precise) form: f32-level, 1e-6 of sum|a b|
    assert (np.abs(got[:, 64:128] - ref[:, 64:128]) <= _bound(dZ, W.T) / 20 + 1e-5).all()
    assert (got[:, 64:128][Y[:, 64:128] <= 0] == 0).all()
    assert np.array_equal(got[:, :64], base[:, :64]) and np.array_equal(got[:, 128:], base[:, 128:])


def _pb(t, off=0):
    return ctypes.c_void_p(t.data_ptr() + 2 * off)


@pytest.mark.parametrize("M,N,K", [(300, 64, 64), (1000, 256, 960), (4096, 128, 128)])
def test_gemm_bf2_is_bitwise_the_f32_staged_gemm(M, N, K):
    """Operands as bf16 hi / lo planes (split once; pcadv_gemm_bf2) give the
    three-product GEMM bit for bit, and the epilogue's own output planes are
    the split of its f32 output."""
    lib = _lib.load()
    rng = np.random.default_rng(M + K)
    A = rng.standard_normal((M, K)).astype(np.float32)
    W = rng.standard_normal((N, K)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    tA, tW, tb = _t(A), _t(W), _t(b)
    ref = torch.empty(M, N, device=DEV)
    check(lib.pcadv_gemm(_p(tA), K, 0, _p(tW), K, 0, _p(ref), N, M, N, K, _p(tb), None, 0, 1, 0,
                         None, 0, 0, None, None, 0, stream_ptr()), "gemm")
    ah, al = torch.empty(M, K, device=DEV, dtype=torch.bfloat16), torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
    wh, wl = torch.empty(N, K, device=DEV, dtype=torch.bfloat16), torch.empty(N, K, device=DEV, dtype=torch.bfloat16)
    check(lib.pcadv_split_bf2(_p(tA), K, M, K, _pb(ah), _pb(al), K, stream_ptr()), "split")
    check(lib.pcadv_split_bf2(_p(tW), K, N, K, _pb(wh), _pb(wl), K, stream_ptr()), "split")
    assert torch.equal(ah.float() + al.float(), (tA.to(torch.bfloat16).float()
                                                 + (tA - tA.to(torch.bfloat16).float()).to(torch.bfloat16).float()))
    C = torch.empty(M, N, device=DEV)
    ch, cl = torch.empty(M, N, device=DEV, dtype=torch.bfloat16), torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    check(lib.pcadv_gemm_bf2(_pb(ah), _pb(al), K, _pb(wh), _pb(wl), K, _p(C), N, _pb(ch), _pb(cl), N,
                             M, N, K, _p(tb), None, 0, 1, 0, None, 0, stream_ptr()), "gemm_bf2")
    assert torch.equal(C, ref)
    assert torch.equal(ch, C.to(torch.bfloat16))
    assert torch.equal(cl, (C - ch.float()).to(torch.bfloat16))


def _with_gemm_big(enabled, fn):
    # PCADV_GEMM_BIG_PLAIN: the 256-tile kernel also where whole 128-tiles would
    # take the LDS-DMA 128-tile kernel, so the plain modes are exercised too
    saved = {k: os.environ.get(k) for k in ("PCADV_GEMM_BIG", "PCADV_GEMM_BIG_PLAIN")}
    os.environ["PCADV_GEMM_BIG"] = "1" if enabled else "0"
    os.environ["PCADV_GEMM_BIG_PLAIN"] = "1"
    try:
        out = fn()
        torch.cuda.synchronize()
        return out
    finally:
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _planes(x):
    lib = _lib.load()
    R, K = x.shape
    hi = torch.empty(R, K, device=DEV, dtype=torch.bfloat16)
    lo = torch.empty(R, K, device=DEV, dtype=torch.bfloat16)
    check(lib.pcadv_split_bf2(_p(x), K, R, K, _pb(hi), _pb(lo), K, stream_ptr()), "split")
    return hi, lo


@pytest.mark.parametrize("M,N,K,acc", [(33000, 512, 80, 0), (32768, 512, 128, 1),
                                       (8192, 2048, 512, 0)])
def test_gemm_bf2_256_tiles_bitwise(M, N, K, acc):
    """The 256 x 256-tile kernel (wide plane GEMMs: >= 256 tiles, N % 256 == 0)
    sums the same MFMAs in the same order as the 128-tile kernel: C, its
    output planes, the bias / per-group bias / mask / accumulate epilogue all
    bitwise equal.  Shapes: ragged last row tile + odd k-tile count, the
    accumulate form with a mask, conv6's 2048 columns."""
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    A = torch.randn(M, K, device=DEV, generator=g)
    W = torch.randn(N, K, device=DEV, generator=g)
    b = torch.randn(N, device=DEV, generator=g)
    rpg = 4096
    br = torch.randn((M + rpg - 1) // rpg, N, device=DEV, generator=g)
    Y = torch.randn(M, N, device=DEV, generator=g)
    base = torch.randn(M, N, device=DEV, generator=g)
    ah, al = _planes(A)
    wh, wl = _planes(W)

    def run():
        C = base.clone()
        ch = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
        cl = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
        check(lib.pcadv_gemm_bf2(_pb(ah), _pb(al), K, _pb(wh), _pb(wl), K, _p(C), N,
                                 _pb(ch), _pb(cl), N, M, N, K, _p(b), _p(br), rpg, 1, acc,
                                 _p(Y) if acc else None, N if acc else 0, stream_ptr()), "gemm_bf2")
        return C, ch, cl

    big = _with_gemm_big(True, run)
    small = _with_gemm_big(False, run)
    for x, y in zip(big, small):
        assert torch.equal(x, y)
    # and the values themselves: within the three-product bound of fp64
    A64, W64 = A.double(), W.double()
    ref = A64 @ W64.T + b.double() + br.double()[torch.arange(M, device=DEV) // rpg]
    if acc:
        ref = ref + base.double()
    ref = ref.clamp_min(0)
    if acc:
        ref = ref * (Y > 0)
    bound = 2e-5 * (A64.abs() @ W64.abs().T) + 2e-6 * (1 + base.double().abs())
    assert ((big[0].double() - ref).abs() <= bound).all()


@pytest.mark.parametrize("M,N,K,acc", [(4096, 256, 960, 0), (8192, 128, 64, 1), (2048, 384, 256, 0)])
def test_gemm_bf2_128_tiles_lds_dma_bitwise(M, N, K, acc):
    """The 128-tile plane GEMM staged by LDS-DMA (whole tiles; PCADV_GEMM_GLDS=0
    keeps register staging): C, its planes and the bias / per-group bias /
    mask / accumulate epilogue bitwise the register-staged kernel's."""
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    A = torch.randn(M, K, device=DEV, generator=g)
    W = torch.randn(N, K, device=DEV, generator=g)
    b = torch.randn(N, device=DEV, generator=g)
    rpg = 1024
    br = torch.randn(M // rpg, N, device=DEV, generator=g)
    Y = torch.randn(M, N, device=DEV, generator=g)
    base = torch.randn(M, N, device=DEV, generator=g)
    ah, al = _planes(A)
    wh, wl = _planes(W)

    def run():
        C = base.clone()
        ch = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
        cl = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
        check(lib.pcadv_gemm_bf2(_pb(ah), _pb(al), K, _pb(wh), _pb(wl), K, _p(C), N,
                                 _pb(ch), _pb(cl), N, M, N, K, _p(b), _p(br), rpg, 1, acc,
                                 _p(Y) if acc else None, N if acc else 0, stream_ptr()), "gemm_bf2")
        torch.cuda.synchronize()
        return C, ch, cl

    saved = os.environ.get("PCADV_GEMM_GLDS")
    try:
        os.environ["PCADV_GEMM_GLDS"] = "1"
        dma = run()
        os.environ["PCADV_GEMM_GLDS"] = "0"
        reg = run()
    finally:
        if saved is None:
            del os.environ["PCADV_GEMM_GLDS"]
        else:
            os.environ["PCADV_GEMM_GLDS"] = saved
    for x, y in zip(dma, reg):
        assert torch.equal(x, y)
    A64, W64 = A.double(), W.double()
    ref = A64 @ W64.T + b.double() + br.double()[torch.arange(M, device=DEV) // rpg]
    if acc:
        ref = ref + base.double()
    ref = ref.clamp_min(0)
    if acc:
        ref = ref * (Y > 0)
    bound = 2e-5 * (A64.abs() @ W64.abs().T) + 2e-6 * (1 + base.double().abs())
    assert ((dma[0].double() - ref).abs() <= bound).all()


def test_conv_max_bf2_256_tiles_bitwise():
    """conv6's screened max on the 256-tile kernel (one top-2 record per
    128-row half) gives gmax / gidx bitwise equal to the 128-tile kernel,
    and the argmax agrees with the fp64 one except at near-ties."""
    lib = _lib.load()
    C, Np, K, O = 4, 2048, 512, 2048
    rng = np.random.default_rng(11)
    x = np.maximum(rng.standard_normal((C * Np, K)), 0).astype(np.float32)
    x[5] = x[700]  # a twin pair inside one cloud: equal values, first index wins
    w = (rng.standard_normal((O, K)) / 22.6).astype(np.float32)
    bias = (rng.standard_normal(O) * 0.05).astype(np.float32)
    tx, tw, tb = _t(x), _t(w), _t(bias)
    xh, xl = _planes(tx)
    whh, wll = _planes(tw)
    nb = lib.pcadv_conv_max_x3_workspace_bytes(C, Np, O)
    ws = torch.empty(nb, device=DEV, dtype=torch.uint8)

    def run():
        gmax = torch.empty(C, O, device=DEV)
        gidx = torch.empty(C, O, device=DEV, dtype=torch.int32)
        check(lib.pcadv_conv_max_bf2(_p(tx), K, _pb(xh), _pb(xl), K, C, Np, K, _p(tw), _pb(whh),
                                     _pb(wll), _p(tb), O, 1, _p(gmax), _p(gidx), _p(ws), nb,
                                     stream_ptr()), "conv_max_bf2")
        return gmax, gidx

    gb, ib = _with_gemm_big(True, run)
    gs, is_ = _with_gemm_big(False, run)
    assert torch.equal(gb, gs) and torch.equal(ib, is_)
    z = x.astype(np.float64).reshape(C, Np, K) @ w.T.astype(np.float64) + bias
    ref = np.maximum(z.max(1), 0)
    assert np.abs(gb.cpu().numpy() - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())
    gi = ib.cpu().numpy()
    bad = (gi != z.argmax(1)) & (ref > 0)
    for c, o in np.argwhere(bad):  # only at near-ties of the f64 values
        top = np.sort(z[c, :, o])[-2:]
        assert top[1] - top[0] <= 1e-5 * np.abs(x[c * Np:(c + 1) * Np] @ w[o]).max()


def test_seg_forward_planes_path_is_bitwise_the_f32_path():
    from adversarial_learning_on_pointclouds_amd import seg as segmod
    torch.manual_seed(4)
    m = PointNetSeg(50).to(DEV)
    params = list(m.parameters())
    pts = torch.rand(2, 700, 3, device=DEV) * 2 - 1
    cls = torch.zeros(2, 1, 16, device=DEV)
    cls[0, 0, 3] = cls[1, 0, 9] = 1
    saved = segmod._PLANES
    try:
        segmod._PLANES = True
        a = seg_forward(pts, cls, params, precision="bf16x3")
        segmod._PLANES = False
        b = seg_forward(pts, cls, params, precision="bf16x3")
    finally:
        segmod._PLANES = saved
    for k in ("xloc", "gmax", "gidx", "h1", "h2", "h3", "logits"):
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("B,N,precision", [(2, 700, "fp32"), (4, 2048, "fp32"), (4, 2048, "bf16x3")])
def test_seg_backward_paired_and_deferred_launches_are_bitwise(B, N, precision):
    """The backward's launch forms: each layer's weight and data gradients as
    one paired launch (_Engine.pair) and the weight gradients' slab sums
    deferred to one launch (pcadv_wgrad_flush) give bitwise the gradients of
    one launch per GEMM and per finishing reduction."""
    from adversarial_learning_on_pointclouds_amd import seg as segmod
    torch.manual_seed(5)
    m = PointNetSeg(50).to(DEV)
    params = list(m.parameters())
    pts = torch.rand(B, N, 3, device=DEV) * 2 - 1
    cls = torch.zeros(B, 1, 16, device=DEV)
    cls[:, 0, 3] = 1
    fw = seg_forward(pts, cls, params, precision=precision)
    dl = torch.randn(B * N, 50, device=DEV) * 1e-3
    saved = segmod._PAIR, segmod._DEFER
    outs = []
    try:
        for pair, defer in ((False, False), (True, False), (False, True), (True, True)):
            segmod._PAIR, segmod._DEFER = pair, defer
            outs.append([g.clone() for g in seg_backward(fw, dl)])
    finally:
        segmod._PAIR, segmod._DEFER = saved
    for got in outs[1:]:
        for k, (x, y) in enumerate(zip(outs[0], got)):
            assert torch.equal(x, y), k


@pytest.mark.parametrize("rows,rpg,O,K", [(300, 100, 96, 40), (32768, 2048, 96, 40),
                                          (32768, 0, 256, 960), (16, 0, 256, 2048),
                                          (4096, 0, 64, 3)])
def test_gemm_weight_grad(rows, rpg, O, K):
    """dW = dZ^T X over fixed-order slabs, with the bias gradient and the
    per-group (per-cloud) sums taken from the staged dZ."""
    lib = _lib.load()
    rng = np.random.default_rng(rows + O)
    dZ = rng.standard_normal((rows, O)).astype(np.float32) * (rng.random((rows, O)) > 0.5)
    X = rng.standard_normal((rows, K)).astype(np.float32)
    dW = torch.empty(O, K, device=DEV)
    db = torch.empty(O, device=DEV)
    G = rows // rpg if rpg else 1
    gs = torch.empty(G, O, device=DEV)
    nb = lib.pcadv_gemm_wgrad_workspace_bytes(rows, O, K, rpg)
    ws = torch.empty(nb, device=DEV, dtype=torch.uint8)
    tdZ, tX = _t(dZ), _t(X)
    args = (_p(tdZ), O, _p(tX), K, rows, O, K, _p(dW), K, _p(db), _p(gs) if rpg else None, rpg, 0,
            _p(ws), nb, stream_ptr())
    check(lib.pcadv_gemm_wgrad(*args), "wgrad")
    ref = dZ.T.astype(np.float64) @ X.astype(np.float64)
    assert (np.abs(dW.cpu().numpy() - ref) <= _bound(dZ.T, X.T) / 20 + 1e-5).all()
    d64 = dZ.astype(np.float64)
    assert np.abs(db.cpu().numpy() - d64.sum(0)).max() <= 1e-5 * max(1.0, np.abs(d64).sum(0).max())
    if rpg:
        rg = d64.reshape(G, rpg, O).sum(1)
        assert np.abs(gs.cpu().numpy() - rg).max() <= 1e-5 * max(1.0, np.abs(d64).sum(0).max())
    a, a_db, a_gs = dW.clone(), db.clone(), gs.clone()
    check(lib.pcadv_gemm_wgrad(*args), "wgrad")
    assert torch.equal(a, dW) and torch.equal(a_db, db)  # fixed-order slabs: bitwise reproducible
    # the one-launch finishing reductions (k_wgrad_finish) against the separate
    # k_slab_sum launches, plain and accumulating: bitwise the same sums
    acc = args[:12] + (1,) + args[13:]
    outs = {}
    for split in ("0", "1"):
        os.environ["PCADV_WGRAD_SPLIT_FINISH"] = split
        try:
            dW.copy_(a), db.copy_(a_db), gs.fill_(0)
            check(lib.pcadv_gemm_wgrad(*args), "wgrad")
            plain = (dW.clone(), db.clone(), gs.clone())
            check(lib.pcadv_gemm_wgrad(*acc), "wgrad accumulate")
            outs[split] = plain + (dW.clone(), db.clone())
        finally:
            del os.environ["PCADV_WGRAD_SPLIT_FINISH"]
    for x, y in zip(outs["0"], outs["1"]):
        assert torch.equal(x, y)
    assert torch.equal(outs["0"][0], a) and torch.equal(outs["0"][1], a_db)
    if rpg:
        assert torch.equal(outs["0"][2], a_gs)


@pytest.mark.parametrize("B,O,K0,K1,acc", [(16, 256, 2048, 16, 0), (3, 70, 5, 0, 1), (16, 256, 2048, 50, 1)])
def test_wgrad_small_matches_f64(B, O, K0, K1, acc):
    """pcadv_wgrad_small (fc1's per-cloud columns): dw[o][k] (+)= sum_b s[b][o] x[b][k]
    in f32 with rows in order; one or two operands per launch, into a wider dw
    with a column offset; tolerance 1e-5 relative to the f64 product."""
    lib = _lib.load()
    rng = np.random.default_rng(B * 7 + K1)
    s = rng.standard_normal((B, O)).astype(np.float32)
    x0 = rng.standard_normal((B, K0)).astype(np.float32)
    x1 = rng.standard_normal((B, max(K1, 1))).astype(np.float32)
    ldo = 3 + K0 + max(K1, 1) + 2
    w0 = rng.standard_normal((O, ldo)).astype(np.float32)
    dW, ds, dx0, dx1 = _t(w0), _t(s), _t(x0), _t(x1)  # held: the launch reads them
    check(lib.pcadv_wgrad_small(_p(ds), O, B, O, _p(dx0), K0, K0, _p(dW, 3),
                                _p(dx1) if K1 else None, K1, K1, _p(dW, 3 + K0) if K1 else None,
                                ldo, acc, stream_ptr()), "pcadv_wgrad_small")
    torch.cuda.synchronize()
    want = w0.astype(np.float64)
    base = want.copy()
    want[:, 3:3 + K0] = acc * base[:, 3:3 + K0] + s.astype(np.float64).T @ x0
    if K1:
        want[:, 3 + K0:3 + K0 + K1] = acc * base[:, 3 + K0:3 + K0 + K1] + s.astype(np.float64).T @ x1[:, :K1]
    got = dW.cpu().numpy()
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5 * np.abs(want).max())
    # columns outside the two jobs untouched
    assert np.array_equal(got[:, :3], w0[:, :3])
    assert np.array_equal(got[:, 3 + K0 + K1:], w0[:, 3 + K0 + K1:])


def _wdesc(dZ, X, rows, O, K, dW, db, gs, rpg, acc, ws, nb):
    return _lib.WgradDesc(_p(dZ), O, _p(X), K, rows, O, K, _p(dW), K, _p(db),
                          _p(gs) if gs is not None else None, rpg, int(acc), _p(ws), nb)


def test_gemm_weight_grad_split_batch_is_bitwise():
    """pcadv_gemm_wgrad_slabs + one pcadv_wgrad_finish over the descriptor
    list: the finishing slab sums of several weight gradients (plain,
    accumulating, with per-group sums, more groups than the batch kernel keeps
    in LDS, and more than one batch of descriptors) give bitwise the results of
    the one-call pcadv_gemm_wgrad.  Nothing is retained between calls: a
    slabs call that is never finished changes nothing that follows."""
    lib = _lib.load()
    shapes = [(300, 100, 96, 40), (32768, 2048, 96, 40), (32768, 0, 256, 960), (16, 0, 256, 2048),
              (4096, 0, 64, 3), (8000, 100, 64, 40)] * 3  # 18 > one batch of 16; 80 groups > 64
    cases = []
    for i, (rows, rpg, O, K) in enumerate(shapes):
        rng = np.random.default_rng(100 + i)
        dZ = _t(rng.standard_normal((rows, O)).astype(np.float32))
        X = _t(rng.standard_normal((rows, K)).astype(np.float32))
        G = rows // rpg if rpg else 1
        nb = lib.pcadv_gemm_wgrad_workspace_bytes(rows, O, K, rpg)
        acc = i % 3 == 2
        init = _t(rng.standard_normal((O, K)).astype(np.float32)), _t(rng.standard_normal(O).astype(np.float32))
        cases.append((rows, rpg, O, K, G, nb, acc, dZ, X, init))

    def run(split):
        outs, keep, fin = [], [], []
        for n, (rows, rpg, O, K, G, nb, acc, dZ, X, (w0, b0)) in enumerate(cases):
            dW, db = w0.clone(), b0.clone()
            # per-group sums asked for on every other grouped case
            gs = torch.zeros(G, O, device=DEV) if rpg and n % 2 == 0 else None
            ws = torch.empty(nb, device=DEV, dtype=torch.uint8)
            keep.append(ws)
            if split:
                d = _wdesc(dZ, X, rows, O, K, dW, db, gs, rpg, acc, ws, nb)
                check(lib.pcadv_gemm_wgrad_slabs(ctypes.byref(d), None, stream_ptr()), "slabs")
                fin.append(d)
            else:
                check(lib.pcadv_gemm_wgrad(_p(dZ), O, _p(X), K, rows, O, K, _p(dW), K, _p(db),
                                           _p(gs) if gs is not None else None, rpg, int(acc),
                                           _p(ws), nb, stream_ptr()), "wgrad")
            outs.append((dW, db, gs))
        if split:
            arr = (_lib.WgradDesc * len(fin))(*fin)
            check(lib.pcadv_wgrad_finish(arr, len(fin), stream_ptr()), "finish")
        torch.cuda.synchronize()
        return outs

    ref = run(False)
    # an abandoned split weight gradient (slabs enqueued, never finished)
    rows, rpg, O, K, G, nb, acc, dZ, X, (w0, b0) = cases[0]
    junk = [torch.empty(nb, device=DEV, dtype=torch.uint8), w0.clone(), b0.clone()]
    d = _wdesc(dZ, X, rows, O, K, junk[1], junk[2], None, rpg, 0, junk[0], nb)
    check(lib.pcadv_gemm_wgrad_slabs(ctypes.byref(d), None, stream_ptr()), "abandoned slabs")
    for a, b in zip(ref, run(True)):
        for x, y in zip(a, b):
            assert (x is None and y is None) or torch.equal(x, y)
    check(lib.pcadv_wgrad_finish(None, 0, stream_ptr()), "finish of an empty list")


def test_gemm_wgrad_slabs_paired_with_data_gradient_is_bitwise():
    """pcadv_gemm_wgrad_slabs with a data-gradient descriptor: the two GEMMs
    in one launch give bitwise the outputs of their own launches (pcadv_gemm,
    pcadv_gemm_wgrad), plain and accumulating, masked, with per-group sums."""
    lib = _lib.load()
    rng = np.random.default_rng(77)
    M, O, K, rpg = 4096, 256, 128, 1024
    dZ = _t(rng.standard_normal((M, O)).astype(np.float32))
    X = _t(rng.standard_normal((M, K)).astype(np.float32))
    W = _t(rng.standard_normal((O, K)).astype(np.float32))
    Y = _t(rng.standard_normal((M, K)).astype(np.float32))
    nb = lib.pcadv_gemm_wgrad_workspace_bytes(M, O, K, rpg)
    for acc in (0, 1):
        c0 = _t(rng.standard_normal((M, K)).astype(np.float32))
        outs = []
        for paired in (False, True):
            dW, db = torch.zeros(O, K, device=DEV), torch.zeros(O, device=DEV)
            gs = torch.zeros(M // rpg, O, device=DEV)
            C = c0.clone()
            ws = torch.empty(nb, device=DEV, dtype=torch.uint8)
            g = _lib.GemmDesc(_p(dZ), O, 0, _p(W), K, 1, _p(C), K, M, K, O, None, None, 0, 0, acc,
                              _p(Y), K, 0, None, None, 0)
            if paired:
                d = _wdesc(dZ, X, M, O, K, dW, db, gs, rpg, 0, ws, nb)
                check(lib.pcadv_gemm_wgrad_slabs(ctypes.byref(d), ctypes.byref(g), stream_ptr()), "pair")
                check(lib.pcadv_wgrad_finish(ctypes.byref(d), 1, stream_ptr()), "finish")
            else:
                check(lib.pcadv_gemm_wgrad(_p(dZ), O, _p(X), K, M, O, K, _p(dW), K, _p(db), _p(gs),
                                           rpg, 0, _p(ws), nb, stream_ptr()), "wgrad")
                check(lib.pcadv_gemm(_p(dZ), O, 0, _p(W), K, 1, _p(C), K, M, K, O, None, None, 0, 0,
                                     acc, _p(Y), K, 0, None, None, 0, stream_ptr()), "gemm")
            torch.cuda.synchronize()
            outs.append((dW, db, gs, C))
        for x, y in zip(*outs):
            assert torch.equal(x, y)


def test_colsum_and_group_colsum():
    lib = _lib.load()
    rng = np.random.default_rng(5)
    M, N = 4096, 77
    X = rng.standard_normal((M, N)).astype(np.float32)
    Y = rng.standard_normal((M, N)).astype(np.float32)
    out = torch.empty(N, device=DEV)
    nb = lib.pcadv_colsum_workspace_bytes(M, N)
    ws = torch.empty(nb, device=DEV, dtype=torch.uint8)
    tX, tY = _t(X), _t(Y)
    check(lib.pcadv_colsum(_p(tX), _p(tY), N, N, M, N, _p(out), 0, _p(ws), nb, stream_ptr()),
          "colsum")
    ref = (X * (Y > 0)).astype(np.float64).sum(0)
    assert np.abs(out.cpu().numpy() - ref).max() < 1e-3
    g = torch.empty(4, N, device=DEV)
    check(lib.pcadv_group_colsum(_p(tX), None, N, N, M, N, 1024, _p(g), stream_ptr()), "gcs")
    ref = X.astype(np.float64).reshape(4, 1024, N).sum(1)
    assert np.abs(g.cpu().numpy() - ref).max() < 1e-3


def _cmx(x, w, b, relu=True):
    lib = _lib.load()
    C, N, K = x.shape
    O = w.shape[0]
    gmax = torch.empty(C, O, device=DEV)
    gidx = torch.empty(C, O, device=DEV, dtype=torch.int32)
    nb = lib.pcadv_conv_max_x3_workspace_bytes(C, N, O)
    ws = torch.empty(nb, device=DEV, dtype=torch.uint8)
    xt = _t(x.reshape(C * N, K))
    tw, tb = _t(w), _t(b)
    check(lib.pcadv_conv_max_x3(_p(xt), K, C, N, K, _p(tw), _p(tb), O, int(relu), _p(gmax),
                                _p(gidx), _p(ws), nb, stream_ptr()), "conv_max_x3")
    torch.cuda.synchronize()
    return gmax.cpu().numpy(), gidx.cpu().numpy(), xt


@pytest.mark.parametrize("C,N", [(2, 2048), (3, 300), (1, 97)])
def test_conv_max_x3_vs_oracle(C, N):
    rng = np.random.default_rng(C * N)
    x = np.maximum(rng.standard_normal((C, N, 512)), 0).astype(np.float32)
    w = (rng.standard_normal((2048, 512)) / 22.6).astype(np.float32)
    b = (rng.standard_normal(2048) * 0.05).astype(np.float32)
    gm, gi, _ = _cmx(x, w, b)
    z = x.astype(np.float64) @ w.T.astype(np.float64) + b          # (C, N, O)
    ref_val = np.maximum(z.max(1), 0)
    assert np.abs(gm - ref_val).max() <= 1e-5 * max(1.0, np.abs(ref_val).max())
    am = z.argmax(1)
    pos = ref_val > 0
    bad = (gi != am) & pos
    for c, o in np.argwhere(bad):  # only at near-ties of the f64 values
        assert abs(z[c, gi[c, o], o] - z[c, am[c, o], o]) <= 1e-5 * max(1.0, abs(z[c, am[c, o], o]))


@pytest.mark.parametrize("relu_x", [0, 1])
def test_conv_max_x3_backward_vs_numpy(relu_x):
    lib = _lib.load()
    rng = np.random.default_rng(9)
    C, N, K, O = 2, 300, 512, 2048
    x = np.maximum(rng.standard_normal((C, N, K)), 0).astype(np.float32)
    w = (rng.standard_normal((O, K)) / 22.6).astype(np.float32)
    b = (rng.standard_normal(O) * 0.05).astype(np.float32)
    gm, gi, xt = _cmx(x, w, b)
    dg = rng.standard_normal((C, O)).astype(np.float32)
    dw = torch.empty(O, K, device=DEV)
    db = torch.empty(O, device=DEV)
    base = rng.standard_normal((C * N, K)).astype(np.float32)
    dx = _t(base)
    tdg, tgm, tgi, tw = _t(dg), _t(gm), _t(gi, torch.int32), _t(w)
    check(lib.pcadv_conv_max_x3_bwd(_p(tdg), _p(tgm), _p(tgi), _p(xt), K, C, N, O, K, _p(tw),
                                    _p(dw), _p(db), _p(dx), K, relu_x, stream_ptr()), "cmx_bwd")
    gp = dg * (gm > 0)
    rdw = np.zeros((O, K))
    rdx = base.astype(np.float64).reshape(C, N, K).copy()
    for c in range(C):
        rdw += gp[c][:, None] * x[c, gi[c]]
        add = np.zeros((N, K))
        np.add.at(add, gi[c], gp[c][:, None] * w)
        rdx[c] += add * (x[c] > 0) if relu_x else add
    assert np.abs(dw.cpu().numpy() - rdw).max() <= 1e-5 * np.abs(rdw).max()
    assert np.abs(db.cpu().numpy() - gp.sum(0)).max() <= 1e-5 * np.abs(gp).sum(0).max()
    assert np.abs(dx.cpu().numpy().reshape(C, N, K) - rdx).max() <= 1e-5 * np.abs(rdx).max()


@pytest.mark.parametrize("pattern", ["hull", "one_point", "sparse"])
def test_conv_max_x3_backward_heavy_points(pattern):
    """The sparse max backward when a few points win most channels (hull
    points of a cloud; every channel on one point) or only a few channels are
    live: the hit list of a 64-point range is cut across the 8 waves and the
    cut points are finished in wave order.  Bitwise reproducible."""
    lib = _lib.load()
    rng = np.random.default_rng({"hull": 1, "one_point": 2, "sparse": 3}[pattern])
    C, N, K, O = 3, 700, 512, 2048
    x = np.maximum(rng.standard_normal((C * N, K)), 0).astype(np.float32)
    w = rng.standard_normal((O, K)).astype(np.float32)
    gm = rng.random((C, O)).astype(np.float32) + 0.1
    if pattern == "hull":
        gi = rng.choice([3, 64, 65, 130, 699], size=(C, O)).astype(np.int32)
    elif pattern == "one_point":
        gi = np.full((C, O), 70, np.int32)
    else:
        gi = rng.integers(0, N, (C, O)).astype(np.int32)
        gm[rng.random((C, O)) < 0.95] = -1.0  # relu'd away
    dg = rng.standard_normal((C, O)).astype(np.float32)
    base = rng.standard_normal((C * N, K)).astype(np.float32)
    tdg, tgm, tgi, tw, tx = _t(dg), _t(gm), _t(gi, torch.int32), _t(w), _t(x)
    outs = []
    for _ in range(2):
        dx = _t(base)
        check(lib.pcadv_conv_max_x3_bwd(_p(tdg), _p(tgm), _p(tgi), _p(tx), K, C, N, O, K, _p(tw),
                                        None, None, _p(dx), K, 1, stream_ptr()), "cmx_bwd")
        outs.append(dx.cpu())
    assert torch.equal(outs[0], outs[1])
    gp = (dg * (gm > 0)).astype(np.float64)
    rdx = base.astype(np.float64).reshape(C, N, K).copy()
    for c in range(C):
        add = np.zeros((N, K))
        np.add.at(add, gi[c], gp[c][:, None] * w)
        rdx[c] += add * (x.reshape(C, N, K)[c] > 0)
    err = np.abs(outs[0].numpy().reshape(C, N, K) - rdx).max()
    assert err <= 1e-5 * np.abs(rdx).max(), err


def test_row_ce_vs_oracle():
    rng = np.random.default_rng(11)
    B, N, C = 3, 500, 50
    lg = rng.standard_normal((B, N, C)).astype(np.float32) * 3
    seg = rng.integers(0, C, (B, N))
    t = _t(lg).requires_grad_(True)
    loss = seg_cross_entropy(t, _t(seg, torch.int64))
    loss.backward()
    rl, rg = onp.seg_cross_entropy(lg, seg)
    assert abs(loss.item() - rl) < 1e-5 * max(1, abs(rl))
    assert np.abs(t.grad.cpu().numpy() - rg).max() <= 1e-6


@pytest.mark.parametrize("M,C,ld", [(32, 40, 40), (200, 64, 64), (1000, 50, 50), (300, 100, 100),
                                    (777, 50, 52)])
def test_row_ce_kernel_forms(M, C, ld):
    """pcadv_row_ce's three kernels against fp64: one wave per row (M <= 256,
    C <= 64, the cls heads), rows staged through LDS (C <= 63), a lane per row
    (wider rows); a strided logits matrix too.  Loss = mean CE * 1, gradient
    (softmax - onehot) * scale / M."""
    lib = _lib.load()
    rng = np.random.default_rng(M + C)
    lg = (rng.standard_normal((M, ld)) * 3).astype(np.float32)
    y = rng.integers(0, C, M)
    tl, ty = _t(lg), _t(y, torch.int64)
    loss = torch.empty(1, device=DEV)
    dl = torch.zeros(M, ld, device=DEV)
    nb = lib.pcadv_row_ce_workspace_bytes(M)
    ws = torch.empty(nb, device=DEV, dtype=torch.uint8)
    scale = 0.7
    check(lib.pcadv_row_ce(_p(tl), ld, _p(ty), M, C, ctypes.c_float(scale), _p(loss), _p(dl),
                           _p(ws), nb, stream_ptr()), "row_ce")
    x = lg[:, :C].astype(np.float64)
    lse = np.log(np.exp(x - x.max(1, keepdims=True)).sum(1)) + x.max(1)
    ref_loss = (lse - x[np.arange(M), y]).mean()
    p = np.exp(x - lse[:, None])
    p[np.arange(M), y] -= 1
    ref_g = p * scale / M
    assert abs(loss.item() - ref_loss) <= 1e-5 * max(1.0, abs(ref_loss))
    g = dl.cpu().numpy()
    assert np.abs(g[:, :C] - ref_g).max() <= 1e-6 * max(1.0, np.abs(ref_g).max())
    assert (g[:, C:] == 0).all()  # the padding columns are not written


def _seg_model(S):
    m = PointNetSeg(50)
    m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in S.items()})
    return m.to(DEV)


def test_seg_forward_golden_g6():
    """PointNetSeg forward vs the reference capture (B=2, N=2048)."""
    fx = load("g6_seg_fwd.npz")
    S = onp.make_params(onp.seg_spec(50), seed=int(fx["s_seed"]))
    pts = np.random.default_rng(int(fx["pts_seed"])).uniform(-1, 1, (2, 2048, 3)).astype(np.float32)
    m = _seg_model(S)
    with torch.no_grad():
        out, g = m(_t(pts), _t(fx["cls"]))
    check_tensor_rel(fx, "gmax", g.cpu().numpy()[:, :, 0], tol=1e-3)
    check_tensor_rel(fx, "out", out.cpu().numpy(), tol=1e-3)


def test_seg_step_golden_g8():
    """run_training_pointnet_seg's step: loss, x_global and every gradient vs the
    reference capture (B=2, N=512)."""
    fx = load("g8_seg_step.npz")
    S = onp.make_params(onp.seg_spec(50), seed=int(fx["s_seed"]))
    B, N = fx["seg"].shape
    pts = np.random.default_rng(int(fx["pts_seed"])).uniform(-1, 1, (B, N, 3)).astype(np.float32)
    m = _seg_model(S)
    logits, g, _ = m.forward_points(_t(pts), _t(fx["cls"]))
    loss = seg_cross_entropy(logits, _t(fx["seg"], torch.int64))
    loss.backward()
    assert abs(loss.item() - float(fx["loss"])) < 1e-4
    check_tensor_rel(fx, "gmax", g.detach().cpu().numpy(), tol=1e-3)
    check_tensor_rel(fx, "logits", logits.detach().cpu().numpy().transpose(0, 2, 1), tol=1e-3)
    for name, p in m.named_parameters():
        check_tensor_l2(fx, "grad." + name, p.grad.cpu().numpy(), tol=2e-3)


def _oracle_cache(fw, pts, cls):
    """The oracle's backward cache built from this forward's own activations."""
    B, N, _ = fw["dims"]
    loc = fw["xloc"].cpu().numpy().reshape(B, N, 960)
    offs = [0, 64, 192, 320, 448, 960]
    xs = [loc[:, :, offs[i]:offs[i + 1]] for i in range(5)] + [None]
    return dict(pts=pts, xs=xs, am=fw["gidx"].cpu().numpy().astype(np.int64),
                g=fw["gmax"].cpu().numpy(), loc=loc, cvec=cls.reshape(B, -1),
                h1=fw["h1"].cpu().numpy().reshape(B, N, 256),
                h2=fw["h2"].cpu().numpy().reshape(B, N, 256),
                h3=fw["h3"].cpu().numpy().reshape(B, N, 128))


def _conv6_argmax_ok(fw, S, tol=1e-5):
    """conv6 + ReLU + max (pointnet.py:301-303): the pooled point of every
    channel with a positive max must be the f64 argmax of the kernel's own
    conv5 activations, except at near-ties (values within tol of the max,
    relative to max(1, |max|)); the pooled value must equal the f64 value there
    to 1e-5.  Returns the number of near-tie substitutions."""
    B, N, _ = fw["dims"]
    x5 = fw["xloc"][:, 448:960].double().reshape(B, N, 512)
    W6 = torch.from_numpy(S["conv6.weight"].reshape(2048, 512)).to(DEV, torch.float64)
    b6 = torch.from_numpy(S["conv6.bias"]).to(DEV, torch.float64)
    gi = fw["gidx"].long()
    near = 0
    for c in range(B):
        y = torch.relu(x5[c] @ W6.T + b6)           # N x 2048
        best, am = y.max(0)
        yg = y.gather(0, gi[c].unsqueeze(0)).squeeze(0)
        pos = best > 0
        lim = tol * torch.clamp(best.abs(), min=1.0)
        assert bool((yg[pos] >= best[pos] - lim[pos]).all()), f"cloud {c}: pooled below the f64 max"
        g = fw["gmax"][c].double()
        assert bool(((g - best).abs() <= lim).all()), f"cloud {c}: pooled value off the f64 max"
        near += int(((gi[c] != am) & pos).sum())
    return near


@pytest.mark.parametrize("B,N", [(3, 700), (2, 2048)])
def test_seg_backward_vs_oracle_same_masks(B, N):
    """The backward (every parameter gradient) against the oracle's backward
    evaluated on this forward's activations: 1e-4 of each tensor's max."""
    S = onp.make_params(onp.seg_spec(50), seed=21 + N)
    rng = np.random.default_rng(22 + N)
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    cls = np.zeros((B, 1, 16), np.float32)
    cls[np.arange(B), 0, rng.integers(0, 16, B)] = 1
    seg = rng.integers(0, 50, (B, N))
    params = [_t(v) for v in S.values()]
    with torch.no_grad():
        fw = seg_forward(_t(pts), _t(cls), params)
        logits = fw["logits"].cpu().numpy().reshape(B, N, 50)
        _, dout = onp.seg_cross_entropy(logits, seg)
        grads = seg_backward(fw, _t(dout.reshape(B * N, 50)))
    ref = onp.seg_backward(S, _oracle_cache(fw, pts, cls), dout)
    for (name, r), g in zip(ref.items(), grads):
        e = np.abs(g.cpu().numpy().reshape(r.shape) - r).max() / max(np.abs(r).max(), 1e-30)
        assert e < 1e-4, (name, e)


def test_seg_backward_more_clouds_than_the_batch_kernel_groups():
    """B = 80 > 64 clouds (fc1's per-cloud sums then have more groups than the
    finishing batch kernel keeps in LDS): the split (slabs + one finish launch)
    and the one-call backward agree bitwise, and both match the oracle's
    backward on this forward's activations (this raised before)."""
    from adversarial_learning_on_pointclouds_amd import seg as segmod
    B, N = 80, 64
    S = onp.make_params(onp.seg_spec(50), seed=91)
    rng = np.random.default_rng(92)
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    cls = np.zeros((B, 1, 16), np.float32)
    cls[np.arange(B), 0, rng.integers(0, 16, B)] = 1
    seg = rng.integers(0, 50, (B, N))
    params = [_t(v) for v in S.values()]
    saved = segmod._PAIR, segmod._DEFER
    outs = []
    try:
        with torch.no_grad():
            fw = seg_forward(_t(pts), _t(cls), params)
            logits = fw["logits"].cpu().numpy().reshape(B, N, 50)
            _, dout = onp.seg_cross_entropy(logits, seg)
            for pair, defer in ((True, True), (False, False)):
                segmod._PAIR, segmod._DEFER = pair, defer
                outs.append([g.clone() for g in seg_backward(fw, _t(dout.reshape(B * N, 50)))])
    finally:
        segmod._PAIR, segmod._DEFER = saved
    for x, y in zip(*outs):
        assert torch.equal(x, y)
    ref = onp.seg_backward(S, _oracle_cache(fw, pts, cls), dout)
    for (name, r), g in zip(ref.items(), outs[0]):
        e = np.abs(g.cpu().numpy().reshape(r.shape) - r).max() / max(np.abs(r).max(), 1e-30)
        assert e < 1e-4, (name, e)


def test_seg_step_vs_oracle_ragged():
    """B=3, N=700 (a ragged last tile) end to end vs the numpy oracle."""
    S = onp.make_params(onp.seg_spec(50), seed=21)
    rng = np.random.default_rng(22)
    B, N = 3, 700
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    cls = np.zeros((B, 1, 16), np.float32)
    cls[np.arange(B), 0, rng.integers(0, 16, B)] = 1
    seg = rng.integers(0, 50, (B, N))
    m = _seg_model(S)
    logits, g, gi = m.forward_points(_t(pts), _t(cls))
    loss = seg_cross_entropy(logits, _t(seg, torch.int64))
    loss.backward()
    rl, grads, rlog, rg, ram = onp.seg_step(S, pts, cls, seg)
    assert abs(loss.item() - rl) < 1e-4
    e = np.abs(logits.detach().cpu().numpy() - rlog).max() / np.abs(rlog).max()
    assert e < 1e-3, e
    e = np.abs(g.detach().cpu().numpy() - rg).max() / np.abs(rg).max()
    assert e < 1e-3, e
    gi = gi.cpu().numpy()
    assert ((gi == ram) | (rg <= 0)).all()  # argmax of every positive pooled channel
    for name, p in m.named_parameters():
        a, r = p.grad.cpu().numpy(), grads[name]
        e = np.linalg.norm(a - r) / max(np.linalg.norm(r), 1e-30)
        assert e < 2e-3, (name, e)


def test_seg_deterministic():
    S = onp.make_params(onp.seg_spec(50), seed=23)
    rng = np.random.default_rng(24)
    pts = _t(rng.uniform(-1, 1, (2, 1024, 3)).astype(np.float32))
    cls = _t(np.eye(16, dtype=np.float32)[[1, 5]].reshape(2, 1, 16))
    seg = _t(rng.integers(0, 50, (2, 1024)), torch.int64)
    out = []
    for _ in range(2):
        m = _seg_model(S)
        lg, _, _ = m.forward_points(pts, cls)
        seg_cross_entropy(lg, seg).backward()
        out.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]))
    assert torch.equal(out[0], out[1])


def test_seg_train_step_matches_autograd_and_graph():
    """SegTrainStep (native CE + backward into the flat gradient buffer + one
    Adam launch) equals the module's autograd path, and its HIP-graph replay
    equals the eager step bitwise."""
    from adversarial_learning_on_pointclouds_amd.seg import SegTrainStep
    S = onp.make_params(onp.seg_spec(50), seed=31)
    rng = np.random.default_rng(32)
    B, N = 2, 1024
    pts = _t(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32))
    cls = _t(np.eye(16, dtype=np.float32)[[2, 9]].reshape(B, 1, 16))
    seg = _t(rng.integers(0, 50, (B, N)), torch.int64)
    m_ref = _seg_model(S)
    lg, _, _ = m_ref.forward_points(pts, cls)
    l_ref = seg_cross_entropy(lg, seg)
    l_ref.backward()
    m = _seg_model(S)
    step = SegTrainStep(m, device=DEV)
    loss = step(pts, cls, seg, apply_adam=False).item()
    assert abs(loss - l_ref.item()) < 1e-6
    for (name, p), (_, q) in zip(m.named_parameters(), m_ref.named_parameters()):
        assert torch.equal(p.grad, q.grad), name
    # one Adam step vs the oracle's Adam on the same gradients
    g = {k: q.grad.cpu().numpy() for k, q in m_ref.named_parameters()}
    opt = onp.Adam(S)
    opt.step(g)
    step.adam()
    for name, p in m.named_parameters():
        assert np.abs(p.detach().cpu().numpy() - S[name]).max() < 1e-6, name
    # graph replay == eager
    m2 = _seg_model(S)
    st2 = SegTrainStep(m2, device=DEV)
    graph = st2.capture_on(pts, cls, seg)
    m3 = _seg_model(S)
    st3 = SegTrainStep(m3, device=DEV)
    for _ in range(2):
        graph.replay()
        st3(pts, cls, seg)
    torch.cuda.synchronize()
    assert torch.equal(st2.param, st3.param)
    assert torch.equal(st2.loss, st3.loss)


@pytest.mark.parametrize("precision,e2e", [("fp32", 2e-3), ("bf16x3", 1e-2)])
def test_seg_train_step_full_size_configs3_vs_oracle(precision, e2e):
    """BASELINE configs[3] at full size (B=16, N=2048) through SegTrainStep, the
    bench's path (models/pointnet.py:261-317, utils/trainer.py:334-349): loss,
    logits and x_global vs the numpy oracle; conv6's argmax exact except at
    proven near-ties (_conv6_argmax_ok); every gradient vs the oracle's
    backward on this forward's own activations (1e-4 of each tensor's max) and
    end to end in relative L2 (2e-3 in fp32 mode; the labelled bf16x3 mode's
    three-product forward flips more ReLUs: 1e-2); one Adam step vs the
    oracle's Adam on the same gradients."""
    from adversarial_learning_on_pointclouds_amd.seg import SegTrainStep
    from golden_util import assert_grad_close
    B, N = 16, 2048
    S = onp.make_params(onp.seg_spec(50), seed=41)
    rng = np.random.default_rng(42)
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    cls = np.zeros((B, 1, 16), np.float32)
    cls[np.arange(B), 0, rng.integers(0, 16, B)] = 1
    seg = rng.integers(0, 50, (B, N))
    m = _seg_model(S)
    step = SegTrainStep(m, device=DEV, keep_activations=True, precision=precision)
    loss = step(_t(pts), _t(cls), _t(seg, torch.int64), apply_adam=False).item()
    fw = step.fw
    rl, grads, rlog, rg, ram = onp.seg_step(S, pts, cls, seg)
    assert abs(loss - rl) < 1e-4 * max(1.0, abs(rl)), (loss, rl)
    logits = fw["logits"].cpu().numpy().reshape(B, N, 50)
    e = np.abs(logits - rlog).max() / np.abs(rlog).max()
    assert e < 1e-3, e
    g = fw["gmax"].cpu().numpy()
    assert np.abs(g - rg).max() / np.abs(rg).max() < 1e-3
    _conv6_argmax_ok(fw, S)
    # same-mask backward: the oracle's backward on this forward's activations
    _, dout = onp.seg_cross_entropy(logits, seg)
    ref = onp.seg_backward(S, _oracle_cache(fw, pts, cls), dout)
    for name, p in m.named_parameters():
        r = ref[name]
        assert_grad_close(p.grad.cpu().numpy().reshape(r.shape), r, name, 1e-4, 1e-4)
    # end to end against the oracle's own forward (its own ReLU masks)
    for name, p in m.named_parameters():
        r = grads[name]
        a = p.grad.cpu().numpy().reshape(r.shape)
        el2 = np.linalg.norm(a - r) / max(np.linalg.norm(r), 1e-30)
        assert el2 < e2e, (name, el2)
    gnp = {k: q.grad.cpu().numpy() for k, q in m.named_parameters()}
    onp.Adam(S).step(gnp)
    step.adam()
    for name, p in m.named_parameters():
        assert np.abs(p.detach().cpu().numpy() - S[name]).max() < 1e-6, name


@pytest.mark.parametrize("M,N,K,ldb,rows", [(700, 128, 64, 64, 0), (2048, 256, 960, 3024, 1024),
                                            (4096, 50, 128, 128, 0), (333, 512, 128, 128, 0)])
def test_gemm_b3_is_bitwise_the_precise_gemm(M, N, K, ldb, rows):
    """pcadv_gemm_b3 (B as the hi / mid / lo planes pcadv_split_bf3 makes once)
    against pcadv_gemm with precise = 1 (B split three ways per tile): the same
    planes in LDS, the same MFMAs, so C is bitwise equal; ragged M and N, fc1's
    960 local columns of a 3024-wide weight, and a per-cloud bias."""
    from adversarial_learning_on_pointclouds_amd import seg as segmod
    E = segmod._engine()
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g).to(DEV)
    w = (torch.randn(N, ldb, generator=g) * 0.1).to(DEV)
    bias = None if rows else torch.randn(N, generator=g).to(DEV)
    brow = torch.randn((M + rows - 1) // rows, N, generator=g).to(DEV) if rows else None
    hi, mid, lo = (torch.empty(N, ldb, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    E.split3(w, hi, mid, lo)
    c1 = torch.empty(M, N, device=DEV)
    c2 = torch.empty(M, N, device=DEV)
    E.gemm(a, K, w, ldb, c1, N, M, N, K, bias=bias, bias_rows=brow, rows_per_group=rows,
           relu=True, precise=True)
    E.gemm_b3(a, K, (hi, mid, lo), ldb, c2, N, M, N, K, bias=bias, bias_rows=brow,
              rows_per_group=rows, relu=True)
    torch.cuda.synchronize()
    assert torch.equal(c1, c2)
    # the planes: hi / mid are the two-way split's hi / lo, and hi + mid + lo = w
    h2, l2 = torch.empty_like(hi), torch.empty_like(hi)
    E.split(w, h2, l2)
    assert torch.equal(hi, h2) and torch.equal(mid, l2)
    assert torch.equal(hi.float() + mid.float() + lo.float(), w)


def test_seg_step_weight_planes_path_is_bitwise():
    """SegTrainStep in fp32 mode with the forward GEMMs' weights split once per
    step (PCADV_SEG_B3, the default) against the per-tile split: two steps give
    bitwise the same loss, parameters and gradients."""
    from adversarial_learning_on_pointclouds_amd import seg as segmod
    torch.manual_seed(6)
    res = []
    saved = segmod._B3
    try:
        for b3 in (True, False):
            segmod._B3 = b3
            m = PointNetSeg(50).to(DEV)
            torch.manual_seed(7)
            m.load_state_dict({k: torch.randn_like(v) * 0.1 for k, v in m.state_dict().items()})
            st = segmod.SegTrainStep(m, lr=1e-3)
            pts = torch.rand(4, 2048, 3, device=DEV) * 2 - 1
            cls = torch.zeros(4, 1, 16, device=DEV)
            cls[:, 0, 5] = 1
            lab = torch.randint(0, 50, (4, 2048), device=DEV)
            losses = [st(pts, cls, lab).clone() for _ in range(2)]
            res.append((losses, st.param.clone(), st.grad.clone()))
    finally:
        segmod._B3 = saved
    (la, pa, ga), (lb, pb, gb) = res
    assert all(torch.equal(x, y) for x, y in zip(la, lb))
    assert torch.equal(pa, pb) and torch.equal(ga, gb)
