"""numpy fp32 restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).

Every function names the reference lines it restates (paths relative to the
reference repository root).  Layouts are point-major: a cloud batch is
``(B, N, C)`` with channels contiguous, which is the transpose of the
reference's ``B x C x N`` Conv1d layout; weights keep the reference's
``[out, in(, 1)]`` state-dict shapes.

The max-pool backward is the sparse form (gradient routed to the first argmax
point of each channel), which equals torch's dense ``MaxBackward`` whenever
the maximum is unique (``models/pointnet.py:129``).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import scipy.sparse as _sparse

F32 = np.float32

# --------------------------------------------------------------------------
# parameter specs: reference state_dict names and shapes
# --------------------------------------------------------------------------

# models/pointnet.py:186-195 (PointNetCls(k=40, feature_transform=False)) +
# :81-94 (PointNetfeat); cls factory utils/model_utils.py:68-70.
def cls_spec(k: int = 40):
    return [
        ("feat.conv1.weight", (64, 3, 1)), ("feat.conv1.bias", (64,)),
        ("feat.conv2.weight", (64, 64, 1)), ("feat.conv2.bias", (64,)),
        ("feat.conv3.weight", (128, 64, 1)), ("feat.conv3.bias", (128,)),
        ("feat.conv4.weight", (1024, 128, 1)), ("feat.conv4.bias", (1024,)),
        ("fc1.weight", (512, 1024)), ("fc1.bias", (512,)),
        ("fc2.weight", (256, 512)), ("fc2.bias", (256,)),
        ("fc3.weight", (k, 256)), ("fc3.bias", (k,)),
    ]


# models/pointnet.py:46-57 (STNkd); STN3d is stnkd_spec(3) with fc3 -> 9.
def stnkd_spec(prefix: str, k: int):
    return [
        (prefix + "conv1.weight", (64, k, 1)), (prefix + "conv1.bias", (64,)),
        (prefix + "conv2.weight", (128, 64, 1)), (prefix + "conv2.bias", (128,)),
        (prefix + "conv3.weight", (1024, 128, 1)), (prefix + "conv3.bias", (1024,)),
        (prefix + "fc1.weight", (512, 1024)), (prefix + "fc1.bias", (512,)),
        (prefix + "fc2.weight", (256, 512)), (prefix + "fc2.bias", (256,)),
        (prefix + "fc3.weight", (k * k, 256)), (prefix + "fc3.bias", (k * k,)),
    ]


def cls_ft_spec(k: int = 40):
    """PointNetCls(k, feature_transform=True): feat.fstn = STNkd(64) is
    registered after feat.conv1..conv4 (models/pointnet.py:86-94)."""
    s = cls_spec(k)
    return s[:8] + stnkd_spec("feat.fstn.", 64) + s[8:]


# models/discriminator.py:30-39 (DeepConvDiscNet(input_dim, output_dim)).
def disc_spec(input_dim: int = 40, output_dim: int = 1):
    return [
        ("conv1.weight", (512, input_dim, 1)), ("conv1.bias", (512,)),
        ("conv2.weight", (256, 512, 1)), ("conv2.bias", (256,)),
        ("conv3.weight", (256, 256, 1)), ("conv3.bias", (256,)),
        ("conv4.weight", (64, 256, 1)), ("conv4.bias", (64,)),
        ("conv5.weight", (64, 64, 1)), ("conv5.bias", (64,)),
        ("fc.weight", (output_dim, 64)), ("fc.bias", (output_dim,)),
    ]


# models/pointnet.py:261-278 (PointNetSeg(NUM_SEG_CLASSES)).
def seg_spec(num_seg_classes: int = 50):
    dims = [(64, 3), (128, 64), (128, 128), (128, 128), (512, 128), (2048, 512)]
    s = []
    for i, (o, c) in enumerate(dims, 1):
        s += [(f"conv{i}.weight", (o, c, 1)), (f"conv{i}.bias", (o,))]
    s += [("fc1.weight", (256, 3024)), ("fc1.bias", (256,)),
          ("fc2.weight", (256, 256)), ("fc2.bias", (256,)),
          ("fc3.weight", (128, 256)), ("fc3.bias", (128,)),
          ("fc4.weight", (num_seg_classes, 128)), ("fc4.bias", (num_seg_classes,))]
    return s


def _fans(shape):
    fan_in = int(np.prod(shape[1:]))
    return fan_in, int(shape[0]) * int(np.prod(shape[2:]))


def make_params(spec, seed: int, init: str = "default") -> "OrderedDict[str, np.ndarray]":
    """Deterministic weights from numpy PCG64 (stable across numpy versions).

    ``init="default"`` mirrors the bounds of torch's default Conv1d/Linear init
    (U(+-1/sqrt(fan_in)) for weight and bias; PointNetCls is built with it,
    utils/model_utils.py:68-70).  ``init="xavier"`` mirrors
    utils/model_utils.py:27-58 with init_type='xavier' (xavier_normal gain 1,
    bias 0), used for the discriminator (:104-106).
    """
    rng = np.random.default_rng(seed)
    out = OrderedDict()
    last_fan_in = None
    for name, shape in spec:
        if name.endswith("weight"):
            fan_in, fan_out = _fans(shape)
            last_fan_in = fan_in
            if init == "xavier":
                std = math.sqrt(2.0 / (fan_in + fan_out))
                out[name] = rng.normal(0.0, std, shape).astype(F32)
            else:
                b = 1.0 / math.sqrt(fan_in)
                out[name] = rng.uniform(-b, b, shape).astype(F32)
        else:
            if init == "xavier":
                out[name] = np.zeros(shape, F32)
            else:
                b = 1.0 / math.sqrt(last_fan_in)
                out[name] = rng.uniform(-b, b, shape).astype(F32)
    return out


def _w(p, name):
    w = p[name]
    return w.reshape(w.shape[0], -1) if w.ndim == 3 else w


def relu(x):
    return np.maximum(x, F32(0))


# --------------------------------------------------------------------------
# generator: PointNetCls
# --------------------------------------------------------------------------

def bf16_round(a):
    """Round an f32 array to bfloat16 (nearest, ties to even), returned as f32:
    the operand rounding of the build's bf16 mode (a bf16 MFMA input)."""
    u = np.ascontiguousarray(a, F32).view(np.uint32)
    r = (u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) & np.uint32(0xFFFF0000)
    return r.view(F32)


def point_mlp_fwd(pts, p, prefix="feat.", precision="fp32"):
    """relu(conv1), relu(conv2), relu(conv3) as per-point matvecs
    (models/pointnet.py:115-116,127).  pts: (B, N, 3).  precision "bf16" (the
    build's bf16 mode, not a reference behaviour): conv3's inputs and weights
    rounded to bf16, the products summed exactly (f64) and rounded to f32, and
    the activation x3 kept in bf16 (rounded once more: what conv4 and the
    backward read)."""
    def layer(x, i):
        w = _w(p, f"{prefix}conv{i}.weight")
        if precision == "bf16" and i == 3:
            y = (bf16_round(x).astype(np.float64) @ bf16_round(w).astype(np.float64).T).astype(F32)
        else:
            y = x @ w.T
        y += p[f"{prefix}conv{i}.bias"]
        return np.maximum(y, F32(0), out=y)
    x1 = layer(pts, 1)
    x2 = layer(x1, 2)
    x3 = layer(x2, 3)
    if precision == "bf16":
        x3 = bf16_round(x3)
    return x1, x2, x3


def conv_max_fwd(x, w, b, relu_before_max=False, precision="fp32"):
    """conv (1x1) then max over points, first index on ties
    (models/pointnet.py:128-130; torch.max(dim) returns the first maximal index
    on CPU).  x: (B, N, K), w: (O, K).  Returns (gmax (B, O), argmax (B, O)).
    precision "bf16": the conv on bf16-rounded x and w, products summed in f64."""
    B = x.shape[0]
    O = w.shape[0]
    N, K = x.shape[1], x.shape[2]
    # channel-major (O, B, N) from one GEMM, so the argmax runs along contiguous memory
    if precision == "bf16":
        y = (bf16_round(w).astype(np.float64) @ bf16_round(x.reshape(B * N, K)).astype(np.float64).T
             ).astype(F32)
    else:
        y = w @ x.reshape(B * N, K).T
    y += b[:, None]
    if relu_before_max:
        np.maximum(y, F32(0), out=y)
    y = y.reshape(O, B, N)
    am = np.argmax(y, axis=2).T.astype(np.int32)                 # (B, O)
    gmax = y[np.arange(O)[None, :], np.arange(B)[:, None], am].astype(F32)
    return gmax, am


def head_fwd(g, p, mask=None, p_drop=0.3):
    """relu(fc1) -> relu(dropout(fc2)) -> fc3 (models/pointnet.py:200-202).
    ``mask`` (B, 256) of {0,1} replaces nn.Dropout's Bernoulli draw; eval mode
    passes None."""
    h1 = relu(g @ p["fc1.weight"].T + p["fc1.bias"]).astype(F32)
    z2 = (h1 @ p["fc2.weight"].T + p["fc2.bias"]).astype(F32)
    scale = None
    if mask is not None:
        scale = (mask.astype(F32) * (F32(1.0) / F32(1.0 - p_drop))).astype(F32)
        z2 = z2 * scale
    h2 = relu(z2).astype(F32)
    logits = (h2 @ p["fc3.weight"].T + p["fc3.bias"]).astype(F32)
    return logits, (h1, h2, scale)


def cls_forward(p, pts, mask=None, precision="fp32"):
    """PointNetCls.forward (models/pointnet.py:197-203), feature_transform=False.
    Returns logits (B, k), global (B, 1024) and a cache for cls_backward.
    precision "bf16": conv3 / conv4 as in point_mlp_fwd / conv_max_fwd (the
    backward stays f32 on those activations)."""
    pts = np.ascontiguousarray(pts, F32)
    x1, x2, x3 = point_mlp_fwd(pts, p, precision=precision)
    gmax, am = conv_max_fwd(x3, _w(p, "feat.conv4.weight"), p["feat.conv4.bias"],
                            precision=precision)
    logits, hc = head_fwd(gmax, p, mask)
    cache = dict(pts=pts, x1=x1, x2=x2, x3=x3, gmax=gmax, am=am, head=hc)
    return logits, gmax, cache


def conv_max_bwd(dg, am, x, w):
    """Sparse MaxBackward + conv backward (models/pointnet.py:128-129):
    dW[o,:] = sum_b dg[b,o] x[b, am[b,o], :], db = sum_b dg, and
    dX[b, am[b,o], :] += dg[b,o] * W[o,:]."""
    B, N, K = x.shape
    O = w.shape[0]
    rows = x[np.arange(B)[:, None], am]                      # (B, O, K)
    dW = np.einsum("bo,bok->ok", dg, rows)
    # scatter-add of dg[b,o] * W[o,:] onto point am[b,o] as a sparse product
    # (one entry per column; each row sums its entries in ascending o)
    M = _sparse.csr_matrix((dg.reshape(-1), ((np.arange(B)[:, None] * N + am).reshape(-1),
                                             np.arange(B * O))), shape=(B * N, B * O))
    dX = np.asarray(M @ np.tile(w, (B, 1)), dtype=F32).reshape(B, N, K)
    return dW.astype(F32), dg.sum(0).astype(F32), dX


def conv_max_bwd_dense(dg, am, x, w):
    """conv_max_bwd as the reference's autograd computes it (models/pointnet.py:
    128-129 under loss.backward(), utils/trainer.py:520): MaxBackward zero-fills
    the whole (B, N, O) conv4 output gradient and scatters dg at the argmax
    points, then the Conv1d backward runs its two dense GEMMs over all B*N
    points (dX = dY W, dW = dY^T X).  Same values as the sparse form (up to
    summation order); used only to time the reference's algorithm (bench.py's
    cpu_baseline), never as a checker."""
    B, N, K = x.shape
    O = w.shape[0]
    dY = np.zeros((B, N, O), F32)
    dY[np.arange(B)[:, None], am, np.arange(O)[None, :]] = dg
    dY2 = dY.reshape(B * N, O)
    dX = np.matmul(dY, w)  # per cloud, as the Conv1d backward batches it
    dW = dY2.T @ x.reshape(B * N, K)
    return dW.astype(F32), dY2.sum(0).astype(F32), dX.astype(F32)


def cls_backward(p, cache, dlogits, dense_max_bwd=False):
    """Autograd of cls_forward given dL/dlogits; returns grads keyed like the
    reference state_dict (conv weights shaped [out, in, 1]).  dense_max_bwd:
    conv4 + max backward in the reference's dense form (conv_max_bwd_dense:
    timing of the reference algorithm only)."""
    pts, x1, x2, x3 = cache["pts"], cache["x1"], cache["x2"], cache["x3"]
    gmax, am = cache["gmax"], cache["am"]
    h1, h2, scale = cache["head"]
    g = OrderedDict()
    dlogits = dlogits.astype(F32)
    g["fc3.weight"] = dlogits.T @ h2
    g["fc3.bias"] = dlogits.sum(0)
    dz2 = (dlogits @ p["fc3.weight"]) * (h2 > 0)
    if scale is not None:
        dz2 = dz2 * scale
    g["fc2.weight"] = dz2.T @ h1
    g["fc2.bias"] = dz2.sum(0)
    dz1 = (dz2 @ p["fc2.weight"]) * (h1 > 0)
    g["fc1.weight"] = dz1.T @ gmax
    g["fc1.bias"] = dz1.sum(0)
    dgl = (dz1 @ p["fc1.weight"]).astype(F32)
    W4 = _w(p, "feat.conv4.weight")
    dW4, db4, dX3 = (conv_max_bwd_dense if dense_max_bwd else conv_max_bwd)(dgl, am, x3, W4)
    B, N, _ = x3.shape
    dz3 = (dX3 * (x3 > 0)).reshape(B * N, -1)
    dz2p = (dz3 @ _w(p, "feat.conv3.weight")) * (x2.reshape(B * N, -1) > 0)
    dz1p = (dz2p @ _w(p, "feat.conv2.weight")) * (x1.reshape(B * N, -1) > 0)
    feat = OrderedDict()
    feat["feat.conv1.weight"] = (dz1p.T @ pts.reshape(B * N, 3))[:, :, None]
    feat["feat.conv1.bias"] = dz1p.sum(0)
    feat["feat.conv2.weight"] = (dz2p.T @ x1.reshape(B * N, -1))[:, :, None]
    feat["feat.conv2.bias"] = dz2p.sum(0)
    feat["feat.conv3.weight"] = (dz3.T @ x2.reshape(B * N, -1))[:, :, None]
    feat["feat.conv3.bias"] = dz3.sum(0)
    feat["feat.conv4.weight"] = dW4[:, :, None]
    feat["feat.conv4.bias"] = db4
    out = OrderedDict()
    for k in list(feat) + ["fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias",
                           "fc3.weight", "fc3.bias"]:
        out[k] = (feat[k] if k in feat else g[k]).astype(F32)
    out["_dglobal"] = dgl
    return out


# --------------------------------------------------------------------------
# discriminator: DeepConvDiscNet
# --------------------------------------------------------------------------

_DLAYERS = ["conv1", "conv2", "conv3", "conv4", "conv5"]


def lrelu(x, s=F32(0.2)):
    return np.where(x > 0, x, x * s).astype(F32)


def disc_forward(d, x):
    """DeepConvDiscNet.forward (models/discriminator.py:42-51): five 1x1 convs
    with LeakyReLU(0.2) then Linear(64, out).  x: (M, C) -> (M, out)."""
    acts = [x.astype(F32)]
    h = acts[0]
    for l in _DLAYERS:
        h = lrelu(h @ _w(d, l + ".weight").T + d[l + ".bias"])
        acts.append(h)
    out = (h @ d["fc.weight"].T + d["fc.bias"]).astype(F32)
    return out, acts


def disc_backward(d, acts, dout, need_params=True, need_input=True):
    """Autograd of disc_forward.  LeakyReLU backward uses the (in-place) output
    sign, which equals the input sign (discriminator.py:39)."""
    g = OrderedDict()
    dout = dout.astype(F32)
    if need_params:
        g["fc.weight"] = dout.T @ acts[5]
        g["fc.bias"] = dout.sum(0)
    dh = dout @ d["fc.weight"]
    for i in range(5, 0, -1):
        l = _DLAYERS[i - 1]
        dz = np.where(acts[i] > 0, dh, dh * F32(0.2)).astype(F32)
        if need_params:
            g[l + ".weight"] = (dz.T @ acts[i - 1])[:, :, None]
            g[l + ".bias"] = dz.sum(0)
        if i > 1 or need_input:
            dh = dz @ _w(d, l + ".weight")
    out = OrderedDict((k, g[k].astype(F32)) for k, _ in disc_spec(acts[0].shape[1],
                                                                  dout.shape[1])) if need_params else None
    return out, (dh.astype(F32) if need_input else None)


# --------------------------------------------------------------------------
# losses (torch.nn.CrossEntropyLoss / BCEWithLogitsLoss, mean reduction)
# --------------------------------------------------------------------------

def log_softmax(x):
    """F.log_softmax(x, dim=1) (utils/trainer.py:472,492)."""
    m = x.max(1, keepdims=True)
    s = x - m
    return (s - np.log(np.exp(s).sum(1, keepdims=True))).astype(F32)


def log_softmax_bwd(lsm, dy):
    return (dy - np.exp(lsm) * dy.sum(1, keepdims=True)).astype(F32)


def cross_entropy(logits, labels):
    """CrossEntropyLoss() (train_classification.py:199) used at trainer.py:469.
    Returns (loss, dloss/dlogits)."""
    B = logits.shape[0]
    lsm = log_softmax(logits)
    loss = -float(np.mean(lsm[np.arange(B), labels]))
    grad = np.exp(lsm)
    grad[np.arange(B), labels] -= 1.0
    return loss, (grad / F32(B)).astype(F32)


def bce_with_logits(x, y):
    """BCEWithLogitsLoss() (train_classification.py:200) used at
    trainer.py:507,537,553.  Returns (loss, dloss/dx)."""
    x = x.astype(np.float64)
    y = y.astype(np.float64)
    l = np.maximum(x, 0) - x * y + np.log1p(np.exp(-np.abs(x)))
    sig = 1.0 / (1.0 + np.exp(-x))
    return float(l.mean()), ((sig - y) / x.size).astype(F32)


# --------------------------------------------------------------------------
# Adam (torch.optim.Adam, single-tensor path; train_classification.py:110-122)
# --------------------------------------------------------------------------

class Adam:
    def __init__(self, params, lr=1e-4, betas=(0.9, 0.999), eps=1e-8):
        self.p = params
        self.lr, (self.b1, self.b2), self.eps = lr, betas, eps
        self.m = OrderedDict((k, np.zeros_like(v)) for k, v in params.items())
        self.v = OrderedDict((k, np.zeros_like(v)) for k, v in params.items())
        self.t = 0

    def step(self, grads):
        """exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2);
        p.addcdiv_(m, sqrt(v)/sqrt(bc2) + eps, value=-lr/bc1)."""
        self.t += 1
        bc1 = 1.0 - self.b1 ** self.t
        bc2s = math.sqrt(1.0 - self.b2 ** self.t)
        w1 = F32(1.0 - self.b1)
        for k in self.p:
            g = grads[k].astype(F32)
            m, v = self.m[k], self.v[k]
            m += w1 * (g - m)
            v *= F32(self.b2)
            v += F32(1.0 - self.b2) * g * g
            denom = np.sqrt(v) / F32(bc2s) + F32(self.eps)
            self.p[k] -= F32(self.lr / bc1) * (m / denom)


# --------------------------------------------------------------------------
# the adversarial step (utils/trainer.py:426-559)
# --------------------------------------------------------------------------

def semi_ce(logits_ng, d_ng, semi_th):
    """run_training_semi's pseudo-label loss (utils/trainer.py:716-728):
    ignore = D_out <= semi_TH, semi_gt = argmax(pred_nogt) (first index),
    CrossEntropyLoss(ignore_index=255) = mean over the kept rows of
    -log_softmax[semi_gt].  Returns (loss or None, dloss/dlogits, kept ratio)."""
    keep = ~(d_ng[:, 0] <= F32(semi_th))
    kept = int(keep.sum())
    ratio = kept / float(keep.size)
    if kept == 0:
        return None, np.zeros_like(logits_ng), ratio
    am = logits_ng.argmax(1)
    lsm = log_softmax(logits_ng)
    rows = np.nonzero(keep)[0]
    loss = -float(np.mean(lsm[rows, am[rows]].astype(np.float64)))
    grad = np.zeros_like(logits_ng)
    p = np.exp(lsm[rows])
    p[np.arange(rows.size), am[rows]] -= 1.0
    grad[rows] = p / F32(kept)
    return loss, grad.astype(F32), ratio


def adv_step(G, D, optG, optD, pts_gt, labels, pts_nogt, mask_gt, mask_nogt,
             y_gt, y_nogt, lambda_cls=1.0, lambda_adv=0.001, apply_adam=True,
             semi=False, semi_th=0.8, lambda_semi=1.0, dense_max_bwd=False):
    """One run_training iteration (semi=True: one run_training_semi iteration
    past semi_start, utils/trainer.py:611-847).  The stochastic parts are
    inputs: dropout masks (B, 256) for the two G passes and the U(0.7,1.05) /
    U(0,0.305) soft D labels drawn by make_D_label(random=True)
    (utils/utils.py:22-31).  ImagePool(0).query is the identity
    (utils/image_pool.py:35-36).  dense_max_bwd: the conv4 + max backward in
    the reference autograd's dense form (the CPU baseline's timing mode)."""
    logits_gt, _, c_gt = cls_forward(G, pts_gt, mask_gt)             # :468
    l, dce = cross_entropy(logits_gt, labels)                          # :469
    lsm_gt = log_softmax(logits_gt)                                    # :472
    logits_ng, _, c_ng = cls_forward(G, pts_nogt, mask_nogt)           # :490
    lsm_ng = log_softmax(logits_ng)                                    # :492
    d_ng, acts_ng = disc_forward(D, lsm_ng)                            # :499
    loss_adv, dadv = bce_with_logits(d_ng, np.ones_like(d_ng))         # :500-508
    # G backward (:510-520); D frozen -> only the input gradient
    _, dlsm = disc_backward(D, acts_ng, F32(lambda_adv) * dadv, need_params=False)
    dlog_ng = log_softmax_bwd(lsm_ng, dlsm)
    loss_semi, semi_ratio = None, None
    if semi:                                                           # :716-743
        loss_semi, dsemi, semi_ratio = semi_ce(logits_ng, d_ng, semi_th)
        dlog_ng = (dlog_ng + F32(lambda_semi) * dsemi).astype(F32)
    ga = cls_backward(G, c_gt, F32(lambda_cls) * dce, dense_max_bwd)
    gb = cls_backward(G, c_ng, dlog_ng, dense_max_bwd)
    gG = OrderedDict((k, (ga[k] + gb[k]).astype(F32)) for k in G)
    # D backward (:526-556)
    d_gt, acts_gt = disc_forward(D, lsm_gt)
    lD1, d1 = bce_with_logits(d_gt, y_gt)
    lD2, d2 = bce_with_logits(d_ng, y_nogt)
    g1, _ = disc_backward(D, acts_gt, F32(0.5) * d1, need_input=False)
    g2, _ = disc_backward(D, acts_ng, F32(0.5) * d2, need_input=False)
    gD = OrderedDict((k, (g1[k] + g2[k]).astype(F32)) for k in D)
    if apply_adam:
        optG.step(gG)                                                   # :558
        optD.step(gD)                                                   # :559
    losses = dict(loss_cls=l, loss_adv=loss_adv, loss_D=0.5 * lD1 + 0.5 * lD2,
                  loss_D_gt=0.5 * lD1, loss_D_nogt=0.5 * lD2, loss_semi=loss_semi,
                  semi_ratio=semi_ratio)
    aux = dict(logits_gt=logits_gt, logits_nogt=logits_ng, d_nogt=d_ng, d_gt=d_gt,
               am_gt=c_gt["am"], am_nogt=c_ng["am"], gmax_gt=c_gt["gmax"],
               gmax_nogt=c_ng["gmax"])
    return losses, gG, gD, aux


# --------------------------------------------------------------------------
# T-Net path (models/pointnet.py:14-79,118-122,345-353) - forward only
# --------------------------------------------------------------------------

def stn_forward(p, x, prefix, k):
    """STNkd/STN3d forward on point-major x (B, N, k) -> (B, k, k)."""
    h = relu(x @ _w(p, prefix + "conv1.weight").T + p[prefix + "conv1.bias"])
    h = relu(h @ _w(p, prefix + "conv2.weight").T + p[prefix + "conv2.bias"]).astype(F32)
    g, _ = conv_max_fwd(h, _w(p, prefix + "conv3.weight"), p[prefix + "conv3.bias"],
                        relu_before_max=True)
    h = relu(g @ p[prefix + "fc1.weight"].T + p[prefix + "fc1.bias"])
    h = relu(h @ p[prefix + "fc2.weight"].T + p[prefix + "fc2.bias"])
    t = h @ p[prefix + "fc3.weight"].T + p[prefix + "fc3.bias"]
    t = t + np.eye(k, dtype=F32).reshape(1, k * k)
    return t.reshape(-1, k, k).astype(F32)


def cls_ft_forward(p, pts, mask=None):
    """PointNetCls(feature_transform=True).forward (pointnet.py:109-137,197-203)."""
    pts = np.ascontiguousarray(pts, F32)
    x1 = relu(pts @ _w(p, "feat.conv1.weight").T + p["feat.conv1.bias"])
    x2 = relu(x1 @ _w(p, "feat.conv2.weight").T + p["feat.conv2.bias"]).astype(F32)
    trans = stn_forward(p, x2, "feat.fstn.", 64)
    x2t = np.matmul(x2, trans).astype(F32)
    x3 = relu(x2t @ _w(p, "feat.conv3.weight").T + p["feat.conv3.bias"]).astype(F32)
    gmax, am = conv_max_fwd(x3, _w(p, "feat.conv4.weight"), p["feat.conv4.bias"])
    logits, _ = head_fwd(gmax, p, mask)
    return logits, gmax, trans


def feature_transform_regularizer(trans):
    """mean_b ||T T^T - I||_F (models/pointnet.py:345-353)."""
    d = trans.shape[1]
    r = np.matmul(trans, trans.transpose(0, 2, 1)) - np.eye(d, dtype=F32)[None]
    return float(np.mean(np.sqrt((r.astype(np.float64) ** 2).sum((1, 2)))))


def _layer_bwd(dy, x, y, w):
    """Backward of y = relu(x w^T + b) over rows (point-major): returns
    (dW, db, dx) given dL/dy."""
    dz = dy * (y > 0)
    x2 = x.reshape(-1, x.shape[-1])
    dz2 = dz.reshape(-1, dz.shape[-1])
    return (dz2.T @ x2).astype(F32), dz2.sum(0).astype(F32), (dz @ w).astype(F32)


def stn_forward_train(p, x, prefix, k, h1=None, h2=None):
    """STNkd forward keeping what its backward needs (models/pointnet.py:59-79).
    h1 / h2: conv1's / conv2's activations to use instead of recomputing them
    (same-activation checks)."""
    if h1 is None:
        h1 = relu(x @ _w(p, prefix + "conv1.weight").T + p[prefix + "conv1.bias"]).astype(F32)
    if h2 is None:
        h2 = relu(h1 @ _w(p, prefix + "conv2.weight").T + p[prefix + "conv2.bias"]).astype(F32)
    g, am = conv_max_fwd(h2, _w(p, prefix + "conv3.weight"), p[prefix + "conv3.bias"],
                         relu_before_max=True)
    f1 = relu(g @ p[prefix + "fc1.weight"].T + p[prefix + "fc1.bias"]).astype(F32)
    f2 = relu(f1 @ p[prefix + "fc2.weight"].T + p[prefix + "fc2.bias"]).astype(F32)
    t = (f2 @ p[prefix + "fc3.weight"].T + p[prefix + "fc3.bias"]).astype(F32)
    t = t + np.eye(k, dtype=F32).reshape(1, k * k)
    cache = dict(x=x, h1=h1, h2=h2, g=g, am=am, f1=f1, f2=f2)
    return t.reshape(-1, k, k).astype(F32), cache


def stn_backward(p, cache, dT, prefix):
    """Autograd of stn_forward_train given dL/dT (B, k, k): parameter grads and
    dL/dx.  The max-pool follows a ReLU (relu before max, pointnet.py:66-67): the
    argmax point receives the gradient only when the pooled value is > 0."""
    x, h1, h2, g, am, f1, f2 = (cache[n] for n in ("x", "h1", "h2", "g", "am", "f1", "f2"))
    B = x.shape[0]
    out = OrderedDict()
    dt = dT.reshape(B, -1).astype(F32)
    out[prefix + "fc3.weight"] = dt.T @ f2
    out[prefix + "fc3.bias"] = dt.sum(0)
    dz = (dt @ p[prefix + "fc3.weight"]) * (f2 > 0)
    out[prefix + "fc2.weight"] = dz.T @ f1
    out[prefix + "fc2.bias"] = dz.sum(0)
    dz = (dz @ p[prefix + "fc2.weight"]) * (f1 > 0)
    out[prefix + "fc1.weight"] = dz.T @ g
    out[prefix + "fc1.bias"] = dz.sum(0)
    dg = ((dz @ p[prefix + "fc1.weight"]) * (g > 0)).astype(F32)
    W3 = _w(p, prefix + "conv3.weight")
    dW3, db3, dh2 = conv_max_bwd(dg, am, h2, W3)
    out[prefix + "conv3.weight"], out[prefix + "conv3.bias"] = dW3[:, :, None], db3
    dW2, db2, dh1 = _layer_bwd(dh2, h1, h2, _w(p, prefix + "conv2.weight"))
    out[prefix + "conv2.weight"], out[prefix + "conv2.bias"] = dW2[:, :, None], db2
    dW1, db1, dx = _layer_bwd(dh1, x, h1, _w(p, prefix + "conv1.weight"))
    out[prefix + "conv1.weight"], out[prefix + "conv1.bias"] = dW1[:, :, None], db1
    return OrderedDict((k, v.astype(F32)) for k, v in out.items()), dx


def regularizer_bwd(trans):
    """d/dT of mean_b ||T T^T - I||_F: (2 / (B n_b)) (T T^T - I) T."""
    B, d, _ = trans.shape
    a = np.matmul(trans, trans.transpose(0, 2, 1)) - np.eye(d, dtype=F32)[None]
    n = np.sqrt((a.astype(np.float64) ** 2).sum((1, 2)))
    return (np.matmul(a, trans) * (2.0 / (B * n))[:, None, None]).astype(F32)


def conv_max_at(x, w, b, am, relu_before_max=False):
    """conv_max_fwd's pooled values at GIVEN argmax points (a "same activation"
    check feeds the device's own max-pool decisions back into the oracle, so a
    near-tie resolved differently by two f32 summation orders cannot reroute a
    gradient): gmax[b, o] = relu?(x[b, am[b, o]] . w[o] + b[o])."""
    B = x.shape[0]
    rows = x[np.arange(B)[:, None], am]                      # (B, O, K)
    g = (np.einsum("bok,ok->bo", rows, w) + b[None, :]).astype(F32)
    return (np.maximum(g, F32(0)) if relu_before_max else g).astype(F32)


def cls_ft_forward_train(p, pts, mask, am_stn=None, am=None, acts=None):
    """PointNetCls(feature_transform=True).forward in train mode
    (models/pointnet.py:59-79,109-137,197-203) keeping what cls_ft_backward
    needs.  am_stn / am: the STNkd's conv3 and the feature conv4 max-pool
    argmax to use instead of the oracle's own; acts: {"x1", "x2", "h1", "h2",
    "x3"} point-wise activations to use instead of recomputing them (both for
    same-activation checks: a pre-activation within rounding of a ReLU or max
    decision then routes the gradient as the device did)."""
    acts = acts or {}
    pts = np.ascontiguousarray(pts, F32)
    x1 = acts.get("x1")
    if x1 is None:
        x1 = relu(pts @ _w(p, "feat.conv1.weight").T + p["feat.conv1.bias"]).astype(F32)
    x2 = acts.get("x2")
    if x2 is None:
        x2 = relu(x1 @ _w(p, "feat.conv2.weight").T + p["feat.conv2.bias"]).astype(F32)
    trans, sc = stn_forward_train(p, x2, "feat.fstn.", 64, acts.get("h1"), acts.get("h2"))
    if am_stn is not None:
        pre = "feat.fstn."
        g = conv_max_at(sc["h2"], _w(p, pre + "conv3.weight"), p[pre + "conv3.bias"],
                        am_stn, relu_before_max=True)
        f1 = relu(g @ p[pre + "fc1.weight"].T + p[pre + "fc1.bias"]).astype(F32)
        f2 = relu(f1 @ p[pre + "fc2.weight"].T + p[pre + "fc2.bias"]).astype(F32)
        t = (f2 @ p[pre + "fc3.weight"].T + p[pre + "fc3.bias"]).astype(F32)
        t = t + np.eye(64, dtype=F32).reshape(1, 64 * 64)
        trans = t.reshape(-1, 64, 64).astype(F32)
        sc.update(g=g, am=np.asarray(am_stn, np.int64), f1=f1, f2=f2)
    x2t = np.matmul(x2, trans).astype(F32)
    x3 = acts.get("x3")
    if x3 is None:
        x3 = relu(x2t @ _w(p, "feat.conv3.weight").T + p["feat.conv3.bias"]).astype(F32)
    W4 = _w(p, "feat.conv4.weight")
    if am is None:
        gmax, am = conv_max_fwd(x3, W4, p["feat.conv4.bias"])
    else:
        am = np.asarray(am, np.int64)
        gmax = conv_max_at(x3, W4, p["feat.conv4.bias"], am)
    logits, hc = head_fwd(gmax, p, mask)
    cache = dict(pts=pts, x1=x1, x2=x2, trans=trans, sc=sc, x2t=x2t, x3=x3, gmax=gmax, am=am,
                 head=hc)
    return logits, cache


def cls_ft_backward(p, cache, dlogits, lambda_regu=0.0):
    """Autograd of cls_ft_forward_train given dL/dlogits, plus lambda_regu x
    feature_transform_regularizer(trans) (run_training_pointnet_cls adds it,
    utils/trainer.py:257-267; run_training does not, :472-519).  Grads keyed
    and shaped like the state_dict."""
    pts, x1, x2, trans, sc = (cache[n] for n in ("pts", "x1", "x2", "trans", "sc"))
    x2t, x3, gmax, am = cache["x2t"], cache["x3"], cache["gmax"], cache["am"]
    h1, h2, scale = cache["head"]
    g = OrderedDict()
    dl = np.asarray(dlogits, F32)
    g["fc3.weight"] = dl.T @ h2
    g["fc3.bias"] = dl.sum(0)
    dz2 = (dl @ p["fc3.weight"]) * (h2 > 0)
    if scale is not None:
        dz2 = dz2 * scale
    g["fc2.weight"] = dz2.T @ h1
    g["fc2.bias"] = dz2.sum(0)
    dz1 = (dz2 @ p["fc2.weight"]) * (h1 > 0)
    g["fc1.weight"] = dz1.T @ gmax
    g["fc1.bias"] = dz1.sum(0)
    dgl = (dz1 @ p["fc1.weight"]).astype(F32)
    W4 = _w(p, "feat.conv4.weight")
    dW4, db4, dX3 = conv_max_bwd(dgl, am, x3, W4)
    g["feat.conv4.weight"], g["feat.conv4.bias"] = dW4[:, :, None], db4
    dW3, db3, dx2t = _layer_bwd(dX3, x2t, x3, _w(p, "feat.conv3.weight"))
    g["feat.conv3.weight"], g["feat.conv3.bias"] = dW3[:, :, None], db3
    # x2t = x2 @ T (models/pointnet.py:120-121)
    dT = np.matmul(x2.transpose(0, 2, 1), dx2t).astype(F32)
    if lambda_regu:
        dT = dT + F32(lambda_regu) * regularizer_bwd(trans)
    dx2 = np.matmul(dx2t, trans.transpose(0, 2, 1)).astype(F32)
    gs, dx2s = stn_backward(p, sc, dT, "feat.fstn.")
    g.update(gs)
    dx2 = dx2 + dx2s
    dW2, db2, dx1 = _layer_bwd(dx2, x1, x2, _w(p, "feat.conv2.weight"))
    g["feat.conv2.weight"], g["feat.conv2.bias"] = dW2[:, :, None], db2
    dW1, db1, _ = _layer_bwd(dx1, pts, x1, _w(p, "feat.conv1.weight"))
    g["feat.conv1.weight"], g["feat.conv1.bias"] = dW1[:, :, None], db1
    return OrderedDict((k, g[k].astype(F32).reshape(p[k].shape)) for k in p)


def cls_ft_step(p, pts, labels, mask, lambda_cls=1.0, lambda_regu=0.001):
    """One run_training_pointnet_cls iteration body (utils/trainer.py:254-268) for
    PointNetCls(feature_transform=True): loss = lambda_cls * CE + lambda_regu *
    feature_transform_regularizer(trans_feat).  Returns (loss_cls, reg, grads)."""
    logits, c = cls_ft_forward_train(p, pts, mask)
    l, dce = cross_entropy(logits, labels)
    reg = feature_transform_regularizer(c["trans"])
    grads = cls_ft_backward(p, c, (F32(lambda_cls) * dce).astype(F32), lambda_regu)
    aux = dict(logits=logits, gmax=c["gmax"], am=c["am"], trans=c["trans"], am_stn=c["sc"]["am"],
               x2t=c["x2t"], x3=c["x3"])
    return l, reg, grads, aux


def adv_ft_grads(G, D, pts_gt, labels, pts_nogt, mask_gt, mask_nogt, y_gt, y_nogt,
                 lambda_cls=1.0, lambda_adv=0.001, am=None, acts=None):
    """run_training's iteration body (utils/trainer.py:468-556, ImagePool(0))
    with a feature-transform generator: G's and D's gradients before the Adam
    steps.  No regulariser: run_training leaves it commented out (:473-476,
    :511-517).  am: optional (am_stn_gt, am_gt, am_stn_nogt, am_nogt) device
    argmax decisions, acts: (GT, no-GT) activation dicts of cls_ft_forward_train
    (same-activation checks)."""
    am = am or (None, None, None, None)
    acts = acts or (None, None)
    lg, cg = cls_ft_forward_train(G, pts_gt, mask_gt, am[0], am[1], acts[0])  # :467
    l, dce = cross_entropy(lg, labels)                                      # :468
    lsm_gt = log_softmax(lg)                                                # :471
    ln, cn = cls_ft_forward_train(G, pts_nogt, mask_nogt, am[2], am[3], acts[1])  # :490
    lsm_ng = log_softmax(ln)                                                # :492
    d_ng, acts_ng = disc_forward(D, lsm_ng)                                 # :498
    loss_adv, dadv = bce_with_logits(d_ng, np.ones_like(d_ng))              # :499-506
    _, dlsm = disc_backward(D, acts_ng, F32(lambda_adv) * dadv, need_params=False)
    dlog_ng = log_softmax_bwd(lsm_ng, dlsm)
    ga = cls_ft_backward(G, cg, (F32(lambda_cls) * dce).astype(F32))
    gb = cls_ft_backward(G, cn, dlog_ng)
    gG = OrderedDict((k, (ga[k] + gb[k]).astype(F32)) for k in G)
    d_gt, acts_gt = disc_forward(D, lsm_gt)                                 # :526-540
    lD1, d1 = bce_with_logits(d_gt, y_gt)
    lD2, d2 = bce_with_logits(d_ng, y_nogt)                                 # :544-556
    g1, _ = disc_backward(D, acts_gt, F32(0.5) * d1, need_input=False)
    g2, _ = disc_backward(D, acts_ng, F32(0.5) * d2, need_input=False)
    gD = OrderedDict((k, (g1[k] + g2[k]).astype(F32)) for k in D)
    losses = dict(loss_cls=l, loss_adv=loss_adv, loss_D_gt=0.5 * lD1, loss_D_nogt=0.5 * lD2)
    aux = dict(am=(cg["sc"]["am"], cg["am"], cn["sc"]["am"], cn["am"]))
    return losses, gG, gD, aux


# --------------------------------------------------------------------------
# segmentation net (models/pointnet.py:261-317) - forward only
# --------------------------------------------------------------------------

def seg_forward(p, pts, cls):
    """PointNetSeg.forward: pts (B, N, 3), cls (B, 1, 16) -> (B, 50, N), (B, 2048, 1)."""
    pts = np.ascontiguousarray(pts, F32)
    xs = []
    h = pts
    for i in range(1, 7):
        h = relu(h @ _w(p, f"conv{i}.weight").T + p[f"conv{i}.bias"]).astype(F32)
        xs.append(h)
    B, N, _ = pts.shape
    g = xs[5].max(1)                                        # (B, 2048)
    feat = np.concatenate(xs[:5] + [np.broadcast_to(g[:, None, :], (B, N, 2048)),
                                    np.broadcast_to(cls.reshape(B, 1, -1), (B, N, cls.shape[-1]))],
                          axis=2)
    h = relu(feat @ p["fc1.weight"].T + p["fc1.bias"])
    h = relu(h @ p["fc2.weight"].T + p["fc2.bias"])
    h = relu(h @ p["fc3.weight"].T + p["fc3.bias"])
    out = h @ p["fc4.weight"].T + p["fc4.bias"]
    return out.transpose(0, 2, 1).astype(F32), g[:, :, None].astype(F32)


# --------------------------------------------------------------------------
# segmentation training step (models/pointnet.py:282-317 forward + autograd;
# utils/trainer.py:310-400 run_training_pointnet_seg: CrossEntropyLoss over
# every point, pointnet/train_pointnet_seg.py:152; backward; Adam)
# --------------------------------------------------------------------------

def seg_forward_train(p, pts, cls):
    """PointNetSeg.forward keeping what the backward needs.  Returns logits
    (B, N, C) point-major, gmax (B, 2048), and the cache."""
    pts = np.ascontiguousarray(pts, F32)
    B, N, _ = pts.shape
    xs = []
    h = pts
    for i in range(1, 7):
        h = relu(h @ _w(p, f"conv{i}.weight").T + p[f"conv{i}.bias"]).astype(F32)
        xs.append(h)
    x6 = xs[5]
    am = x6.argmax(1)                                        # first index on ties (torch.max)
    g = np.take_along_axis(x6, am[:, None, :], 1)[:, 0, :]   # (B, 2048)
    loc = np.concatenate(xs[:5], axis=2)                     # (B, N, 960) = x1..x5
    W1 = p["fc1.weight"]
    # fc1 over [x1..x5 | tile(gmax) | tile(cls)] (pointnet.py:304-310): the tiled
    # parts are the same for every point of a cloud
    cvec = cls.reshape(B, -1).astype(F32)
    cb = (g @ W1[:, 960:3008].T + cvec @ W1[:, 3008:].T + p["fc1.bias"]).astype(F32)
    h1 = relu(loc @ W1[:, :960].T + cb[:, None, :]).astype(F32)
    h2 = relu(h1 @ p["fc2.weight"].T + p["fc2.bias"]).astype(F32)
    h3 = relu(h2 @ p["fc3.weight"].T + p["fc3.bias"]).astype(F32)
    out = (h3 @ p["fc4.weight"].T + p["fc4.bias"]).astype(F32)
    cache = dict(pts=pts, xs=xs, am=am, g=g, loc=loc, cvec=cvec, h1=h1, h2=h2, h3=h3)
    return out, g, cache


def seg_cross_entropy(logits, seg):
    """CrossEntropyLoss()(pred (B, C, N), seg (B, N)): mean over all B*N points.
    logits point-major (B, N, C).  Returns (loss, dloss/dlogits)."""
    B, N, C = logits.shape
    lsm = log_softmax(logits.reshape(B * N, C))
    lab = seg.reshape(-1)
    loss = -float(np.mean(lsm[np.arange(B * N), lab].astype(np.float64)))
    grad = np.exp(lsm)
    grad[np.arange(B * N), lab] -= 1.0
    return loss, (grad / F32(B * N)).astype(F32).reshape(B, N, C)


def seg_backward(p, cache, dout):
    """Gradients of every PointNetSeg parameter given dL/dlogits (B, N, C)."""
    B, N, _ = dout.shape
    g_ = OrderedDict()

    def lin_bwd(dy, x, name):
        x2 = x.reshape(-1, x.shape[-1])
        d2 = dy.reshape(-1, dy.shape[-1])
        g_[name + ".weight"] = (d2.T @ x2).astype(F32)
        g_[name + ".bias"] = d2.sum(0).astype(F32)

    h1, h2, h3 = cache["h1"], cache["h2"], cache["h3"]
    lin_bwd(dout, h3, "fc4")
    dz = (dout @ p["fc4.weight"]) * (h3 > 0)
    lin_bwd(dz, h2, "fc3")
    dz = (dz @ p["fc3.weight"]) * (h2 > 0)
    lin_bwd(dz, h1, "fc2")
    dz1 = ((dz @ p["fc2.weight"]) * (h1 > 0)).astype(F32)   # (B, N, 256)
    W1 = p["fc1.weight"]
    loc = cache["loc"]
    dW1 = np.zeros_like(W1)
    dW1[:, :960] = dz1.reshape(-1, 256).T @ loc.reshape(-1, 960)
    s1 = dz1.sum(1)                                          # (B, 256): the tiled parts
    dW1[:, 960:3008] = s1.T @ cache["g"]
    dW1[:, 3008:] = s1.T @ cache["cvec"]
    g_["fc1.weight"] = dW1.astype(F32)
    g_["fc1.bias"] = dz1.reshape(-1, 256).sum(0).astype(F32)
    dloc = (dz1 @ W1[:, :960]).astype(F32)                    # (B, N, 960)
    dg = (s1 @ W1[:, 960:3008]).astype(F32)                   # (B, 2048)
    xs = cache["xs"]
    # max over points with the ReLU before it: dg reaches the argmax point
    # when the max is positive (relu'(z) = [x6 > 0] there)
    am = cache["am"]
    w6 = _w(p, "conv6.weight")
    x5 = xs[4]
    act = (cache["g"] > 0).astype(F32)
    dgz = dg * act                                             # (B, 2048)
    dW6 = np.zeros_like(w6)
    dx5_max = np.zeros_like(x5)
    for b in range(B):
        rows = x5[b, am[b]]                                    # (2048, 512)
        dW6 += dgz[b][:, None] * rows
        np.add.at(dx5_max[b], am[b], dgz[b][:, None] * w6)
    g_["conv6.weight"] = dW6.astype(F32)[:, :, None]
    g_["conv6.bias"] = dgz.sum(0).astype(F32)
    offs = [0, 64, 192, 320, 448, 960]
    dy = dx5_max + dloc[:, :, offs[4]:offs[5]]
    for i in range(5, 0, -1):
        x = xs[i - 1]
        xin = xs[i - 2] if i > 1 else cache["pts"]
        dz = (dy * (x > 0)).astype(F32)
        w = _w(p, f"conv{i}.weight")
        g_[f"conv{i}.weight"] = (dz.reshape(-1, dz.shape[-1]).T @ xin.reshape(-1, xin.shape[-1])
                                 ).astype(F32)[:, :, None]
        g_[f"conv{i}.bias"] = dz.reshape(-1, dz.shape[-1]).sum(0).astype(F32)
        if i > 1:
            dy = (dz @ w).astype(F32) + dloc[:, :, offs[i - 2]:offs[i - 1]]
    return OrderedDict((k, g_[k].reshape(p[k].shape).astype(F32)) for k in p)


def seg_step(p, pts, cls, seg, lambda_seg=1.0):
    """One run_training_pointnet_seg iteration's loss and gradients (before
    optimizer.step()).  Returns (loss, grads, logits (B, N, C), gmax, am)."""
    out, g, cache = seg_forward_train(p, pts, cls)
    loss, dout = seg_cross_entropy(out, seg)
    grads = seg_backward(p, cache, (dout * F32(lambda_seg)).astype(F32))
    return loss, grads, out, g, cache["am"]
