"""Tensor-level wrappers of the pcadv HIP kernels + autograd.Functions.

Every wrapper validates shapes, dtypes, devices and contiguity on the host
before launching (a kernel never sees a shape its grid does not assume), then
enqueues on torch's current HIP stream.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import ACT_LRELU, ACT_NONE, ACT_RELU, check, ptr, stream_ptr

__all__ = ["ACT_NONE", "ACT_RELU", "ACT_LRELU", "feat_fwd", "feat_bwd", "conv_max_fwd",
           "conv_max_bwd", "linear_fwd", "linear_bwd", "adam_", "pw_fwd", "pw_bwd_data",
           "pw_bwd_weight", "pw_wgrad_finish", "tnet_reg_fwd", "tnet_reg_bwd", "PointFeatFunction",
           "LinearFunction", "PointwiseFunction", "TransformFunction", "ConvMaxFunction",
           "RegularizerFunction"]


def _req(t, name, shape=None, dtype=torch.float32):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name}: pcadv ops run on the HIP device only (got {t.device})")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
    return t


def _mat(w):
    """Conv1d [out,in,1] or Linear [out,in] weight as a contiguous [out][in]."""
    return w.reshape(w.shape[0], -1)


# ---------------------------------------------------------------------------
# PointNetfeat (feature_transform=False)
# ---------------------------------------------------------------------------

PRECISIONS = {"fp32": 0, "bf16": 1}


def feat_fwd(pts, w1, b1, w2, b2, w3, b3, w4, b4, precision="fp32"):
    """pts (C, N, 3) -> gmax (C, 1024), gidx (C, 1024) int32, x3 (C, N, 128).
    precision "bf16": conv3 / conv4 on bf16-rounded operands (pcadv_feat_fwd_bf16);
    x3 comes back as torch.bfloat16 (the form conv4 and the backward read)."""
    if precision not in PRECISIONS:
        raise ValueError(f"precision {precision!r}: one of {sorted(PRECISIONS)}")
    lib = _lib.load()
    _req(pts, "pts")
    if pts.dim() != 3 or pts.shape[2] != 3:
        raise ValueError(f"pts: expected (C, N, 3), got {tuple(pts.shape)}")
    C, N, _ = pts.shape
    ws = [_req(_mat(w1), "conv1.weight", (64, 3)), _req(b1, "conv1.bias", (64,)),
          _req(_mat(w2), "conv2.weight", (64, 64)), _req(b2, "conv2.bias", (64,)),
          _req(_mat(w3), "conv3.weight", (128, 64)), _req(b3, "conv3.bias", (128,)),
          _req(_mat(w4), "conv4.weight", (1024, 128)), _req(b4, "conv4.bias", (1024,))]
    dev = pts.device
    x3 = torch.empty(C, N, 128, device=dev,
                     dtype=torch.bfloat16 if precision == "bf16" else torch.float32)
    gmax = torch.empty(C, 1024, device=dev)
    gidx = torch.empty(C, 1024, device=dev, dtype=torch.int32)
    nbytes = lib.pcadv_feat_fwd_workspace_bytes(C, N)
    work = torch.empty(nbytes, device=dev, dtype=torch.uint8)
    fn = lib.pcadv_feat_fwd_bf16 if precision == "bf16" else lib.pcadv_feat_fwd
    check(fn(ptr(pts), C, N, *[ptr(t) for t in ws], ptr(x3), ptr(gmax), ptr(gidx),
             ptr(work), nbytes, stream_ptr()), "pcadv_feat_fwd")
    return gmax, gidx, x3


def conv4_max(x3, w4, b4, precision="fp32", out=None):
    """conv4 + max over points of given conv3 activations x3 (C, N, 128) ->
    gmax (C, 1024), gidx (C, 1024) int32: pcadv_feat_fwd's second launch alone
    (pcadv_conv4_max).  A bf16 x3 (feat_fwd's bf16 mode) takes precision
    "bf16" (code 2: the in-step form).  out: optional (gmax, gidx) to write into."""
    if precision not in PRECISIONS:
        raise ValueError(f"precision {precision!r}: one of {sorted(PRECISIONS)}")
    lib = _lib.load()
    code = PRECISIONS[precision]
    if isinstance(x3, torch.Tensor) and x3.dtype == torch.bfloat16:
        if precision != "bf16":
            raise TypeError("x3: a bf16 x3 is bf16 mode's (precision='bf16')")
        _req(x3, "x3", dtype=torch.bfloat16)
        code = 2
    else:
        _req(x3, "x3")
    if x3.dim() != 3 or x3.shape[2] != 128:
        raise ValueError(f"x3: expected (C, N, 128), got {tuple(x3.shape)}")
    C, N, _ = x3.shape
    w = _req(_mat(w4), "conv4.weight", (1024, 128))
    _req(b4, "conv4.bias", (1024,))
    if out is None:
        out = (torch.empty(C, 1024, device=x3.device),
               torch.empty(C, 1024, device=x3.device, dtype=torch.int32))
    gmax, gidx = out
    _req(gmax, "gmax", (C, 1024))
    _req(gidx, "gidx", (C, 1024), torch.int32)
    check(lib.pcadv_conv4_max(ptr(x3), C, N, ptr(w), ptr(b4), ptr(gmax), ptr(gidx),
                              code, stream_ptr()), "pcadv_conv4_max")
    return gmax, gidx


def feat_bwd(dgmax, gidx, pts, w1, b1, w2, b2, w3, w4, x3):
    """Gradients of (conv1..conv4) weights and biases given dL/dgmax.  A bf16
    x3 (feat_fwd's bf16 mode) is widened to f32 first."""
    lib = _lib.load()
    if isinstance(x3, torch.Tensor) and x3.dtype == torch.bfloat16:
        x3 = x3.float()
    C, N, _ = pts.shape
    _req(dgmax, "dgmax", (C, 1024))
    _req(gidx, "gidx", (C, 1024), torch.int32)
    _req(pts, "pts")
    _req(x3, "x3", (C, N, 128))
    mats = [_req(_mat(w1), "conv1.weight", (64, 3)), _req(b1, "conv1.bias", (64,)),
            _req(_mat(w2), "conv2.weight", (64, 64)), _req(b2, "conv2.bias", (64,)),
            _req(_mat(w3), "conv3.weight", (128, 64)), _req(_mat(w4), "conv4.weight", (1024, 128))]
    dev = pts.device
    grads = [torch.empty(64, 3, 1, device=dev), torch.empty(64, device=dev),
             torch.empty(64, 64, 1, device=dev), torch.empty(64, device=dev),
             torch.empty(128, 64, 1, device=dev), torch.empty(128, device=dev),
             torch.empty(1024, 128, 1, device=dev), torch.empty(1024, device=dev)]
    nbytes = lib.pcadv_feat_bwd_workspace_bytes(C, N)
    ws = torch.empty(nbytes, device=dev, dtype=torch.uint8)
    check(lib.pcadv_feat_bwd(ptr(dgmax), ptr(gidx), ptr(pts), C, N, *[ptr(m) for m in mats],
                             ptr(x3), *[ptr(g) for g in grads], ptr(ws), nbytes, stream_ptr()),
          "pcadv_feat_bwd")
    return grads


def conv_max_fwd(x, w, b, relu_before_max=False):
    """x (C, N, 128) point-major; w (O, 128[,1]); -> gmax (C, O), gidx (C, O)."""
    lib = _lib.load()
    _req(x, "x")
    C, N, K = x.shape
    wm = _req(_mat(w), "w")
    O = wm.shape[0]
    _req(b, "b", (O,))
    if wm.shape[1] != K:
        raise ValueError("conv_max_fwd: weight/input width mismatch")
    gmax = torch.empty(C, O, device=x.device)
    gidx = torch.empty(C, O, device=x.device, dtype=torch.int32)
    check(lib.pcadv_conv_max_fwd(ptr(x), C, N, K, ptr(wm), ptr(b), O, int(bool(relu_before_max)),
                                 ptr(gmax), ptr(gidx), stream_ptr()), "pcadv_conv_max_fwd")
    return gmax, gidx


def _out(t, name, like_shape, dev):
    """A caller-given output buffer (e.g. a view of a flat gradient buffer), checked."""
    if t is None:
        return torch.empty(like_shape, device=dev)
    _req(t, name)
    if t.numel() != int(torch.Size(like_shape).numel()):
        raise ValueError(f"{name}: {t.numel()} elements, expected {tuple(like_shape)}")
    return t


def conv_max_bwd(dgmax, gidx, x, w, gmax_relu=None, need_dx=True, dw_out=None, db_out=None,
                 dx_relu=False):
    """Backward of conv_max_fwd: (dx (C, N, K) or None, dw like w, db (O,));
    dw_out / db_out: write the weight gradients there instead; dx_relu: x is a
    ReLU output and dx is returned as dx * [x > 0] (the pre-activation gradient
    of the layer below)."""
    lib = _lib.load()
    _req(x, "x")
    C, N, K = x.shape
    wm = _req(_mat(w), "w")
    O = wm.shape[0]
    _req(dgmax, "dgmax", (C, O))
    _req(gidx, "gidx", (C, O), torch.int32)
    if gmax_relu is not None:
        _req(gmax_relu, "gmax", (C, O))
    dx = torch.empty(C, N, K, device=x.device) if need_dx else None
    dw = _out(dw_out, "dw", tuple(w.shape), x.device)
    db = _out(db_out, "db", (O,), x.device)
    check(lib.pcadv_conv_max_bwd(ptr(dgmax), ptr(gidx), ptr(gmax_relu), ptr(x), C, N, K, ptr(wm),
                                 O, ptr(dw), ptr(db), ptr(dx), int(bool(dx_relu)), stream_ptr()),
          "pcadv_conv_max_bwd")
    return dx, dw, db


# ---------------------------------------------------------------------------
# point-wise layers (rows = points): the feature-transform path
# ---------------------------------------------------------------------------

def _rows(x):
    return x.reshape(-1, x.shape[-1])


def pw_fwd(x, w, b, act, kmajor=False, rows_per_w=0):
    """act(x W^T + b) over the last dim of x (..., K) -> (..., O).  W: Conv1d
    weight [O, K(, 1)], or with kmajor a [K, O] matrix (per rows_per_w rows:
    a (G, K, O) stack, e.g. one transform per cloud)."""
    lib = _lib.load()
    _req(x, "x")
    K = x.shape[-1]
    M = x.numel() // K
    if kmajor:
        _req(w, "w")
        O = w.shape[-1]
    else:
        wm = _req(_mat(w), "w")
        O = wm.shape[0]
    if b is not None:
        _req(b, "b", (O,))
    y = torch.empty(*x.shape[:-1], O, device=x.device)
    check(lib.pcadv_pw_fwd(ptr(x), M, K, ptr(w), ptr(b), O, act, int(bool(kmajor)), rows_per_w,
                           ptr(y), stream_ptr()), "pcadv_pw_fwd")
    return y


def pw_chain(x, layers):
    """Consecutive pw_fwd layers in one launch: layers = [(w, b, act, kmajor,
    rows_per_w), ...], layer i's input the output of layer i-1.  Returns every
    layer's output, bitwise what the per-layer pw_fwd calls return.  Shapes:
    K = 3 -> 64, 64, 64, 128 and K = 64 -> 64, 128 (the feature-transform
    extractor's two runs, include/pcadv.h pcadv_pw_chain)."""
    lib = _lib.load()
    _req(x, "x")
    K = x.shape[-1]
    M = x.numel() // K
    arr = (_lib.PwLayer * len(layers))()
    outs = []
    for i, (w, b, act, kmajor, rows_per_w) in enumerate(layers):
        if kmajor:
            _req(w, "w")
            O = w.shape[-1]
        else:
            O = _req(_mat(w), "w").shape[0]
        if b is not None:
            _req(b, "b", (O,))
        y = torch.empty(*x.shape[:-1], O, device=x.device)
        arr[i] = _lib.PwLayer(ptr(w), ptr(b), ptr(y), O, act, int(bool(kmajor)), rows_per_w)
        outs.append(y)
    check(lib.pcadv_pw_chain(ptr(x), M, K, arr, len(layers), stream_ptr()), "pcadv_pw_chain")
    return outs


def pw_bwd_data(dy, y, act, w, K, kmajor=False, rows_per_w=0, out=None):
    """dx = (dy * act'(y)) W; accumulated into `out` when given."""
    lib = _lib.load()
    _req(dy, "dy")
    O = dy.shape[-1]
    M = dy.numel() // O
    if y is not None:
        _req(y, "y", tuple(dy.shape))
    dx = out if out is not None else torch.empty(*dy.shape[:-1], K, device=dy.device)
    _req(dx, "dx", tuple(dy.shape[:-1]) + (K,))
    check(lib.pcadv_pw_bwd_data(ptr(dy), ptr(y), act, M, O, ptr(w), K, int(bool(kmajor)),
                                rows_per_w, ptr(dx), int(out is not None), stream_ptr()),
          "pcadv_pw_bwd_data")
    return dx


def pw_bwd_weight(dy, y, act, x, rows_per_group=0, kmajor=False, need_db=True, dw_out=None,
                  db_out=None, defer=None):
    """(dW, db) of y = act(x W^T + b): dW (groups, O, K) or kmajor (groups, K, O);
    dw_out / db_out: write them there instead (same element counts).  defer: a
    list; the slab partial sums are left in a workspace and a job appended to
    it, for one pw_wgrad_finish(defer) launch later (dw_out / db_out required,
    rows_per_group 0, [o][k]); returns (dw_out, db_out) unwritten until then."""
    lib = _lib.load()
    _req(dy, "dy")
    _req(x, "x")
    O, K = dy.shape[-1], x.shape[-1]
    M = dy.numel() // O
    if y is not None:
        _req(y, "y", tuple(dy.shape))
    G = rows_per_group if rows_per_group else M
    groups = M // G
    dw = _out(dw_out, "dw", (groups, *((K, O) if kmajor else (O, K))), dy.device)
    db = _out(db_out, "db", (groups, O), dy.device) if need_db else None
    nb = lib.pcadv_pw_bwd_weight_workspace_bytes(M, O, K)
    ws = torch.empty(nb, device=dy.device, dtype=torch.uint8)
    if defer is not None:
        if dw_out is None or rows_per_group or kmajor:
            raise ValueError("pw_bwd_weight(defer=...): dw_out, rows_per_group 0, [o][k]")
        check(lib.pcadv_pw_bwd_weight(ptr(dy), ptr(y), act, ptr(x), M, O, K, 0, 0, None, None,
                                      ptr(ws), nb, stream_ptr()), "pcadv_pw_bwd_weight (slabs)")
        defer.append((_lib.PwWgradJob(ws.data_ptr(), M, O, K, dw.data_ptr(),
                                      db.data_ptr() if db is not None else None), ws))
        return dw, db
    check(lib.pcadv_pw_bwd_weight(ptr(dy), ptr(y), act, ptr(x), M, O, K, rows_per_group,
                                  int(bool(kmajor)), ptr(dw), ptr(db), ptr(ws), nb, stream_ptr()),
          "pcadv_pw_bwd_weight")
    return dw, db


def pw_wgrad_finish(jobs):
    """The slab sums of the weight gradients pw_bwd_weight(defer=jobs) left, in
    one launch (bitwise the per-gradient sums); the workspaces stay alive
    through the list until then."""
    lib = _lib.load()
    arr = (_lib.PwWgradJob * len(jobs))(*[j for j, _ in jobs])
    check(lib.pcadv_pw_wgrad_finish(arr, len(jobs), stream_ptr()), "pcadv_pw_wgrad_finish")


def tnet_reg_fwd(T):
    """feature_transform_regularizer: (reg (), norms (B,))."""
    lib = _lib.load()
    _req(T, "trans")
    B, k, _ = T.shape
    norms = torch.empty(B, device=T.device)
    reg = torch.empty((), device=T.device)
    check(lib.pcadv_tnet_reg_fwd(ptr(T), B, k, ptr(norms), ptr(reg), stream_ptr()),
          "pcadv_tnet_reg_fwd")
    return reg, norms


def tnet_reg_bwd(T, grad_reg):
    lib = _lib.load()
    _req(T, "trans")
    g = _req(grad_reg.reshape(1).contiguous(), "grad")
    B, k, _ = T.shape
    dT = torch.empty_like(T)
    check(lib.pcadv_tnet_reg_bwd(ptr(T), B, k, ptr(g), ptr(dT), stream_ptr()), "pcadv_tnet_reg_bwd")
    return dT


# ---------------------------------------------------------------------------
# linear / 1x1 conv on B x C x 1
# ---------------------------------------------------------------------------

def linear_fwd(x, w, b, act=ACT_NONE, mask=None, p=0.0, add_identity_k=0):
    lib = _lib.load()
    _req(x, "x")
    M, K = x.shape
    wm = _req(_mat(w), "weight")
    Nout = wm.shape[0]
    if wm.shape[1] != K:
        raise ValueError(f"linear: weight {tuple(wm.shape)} does not match input width {K}")
    _req(b, "bias", (Nout,))
    if mask is not None:
        _req(mask, "dropout mask", (M, Nout))
    y = torch.empty(M, Nout, device=x.device)
    check(lib.pcadv_linear_fwd(ptr(x), ptr(wm), ptr(b), ptr(y), M, Nout, K, act, ptr(mask), None,
                               0, float(p), int(add_identity_k), stream_ptr()), "pcadv_linear_fwd")
    return y


def linear_bwd(dy, y, act, mask, p, x, w, need_dx=True, need_dw=True, m_w=None, dw_out=None,
               db_out=None):
    lib = _lib.load()
    M, K = x.shape
    wm = _mat(w)
    Nout = wm.shape[0]
    _req(dy, "grad_output", (M, Nout))
    _req(y, "output", (M, Nout))
    _req(x, "x", (M, K))
    _req(wm, "weight", (Nout, K))
    if mask is not None:
        _req(mask, "dropout mask", (M, Nout))
    m_w = M if m_w is None else m_w
    dx = torch.empty(M, K, device=x.device) if need_dx else None
    dw = _out(dw_out, "weight grad", tuple(w.shape), x.device) if need_dw else None
    db = _out(db_out, "bias grad", (Nout,), x.device) if need_dw else None
    check(lib.pcadv_linear_bwd(ptr(dy), ptr(y), act, ptr(mask), None, 0, float(p), ptr(x), ptr(wm),
                               ptr(dx), ptr(dw), ptr(db), M, m_w, Nout, K, stream_ptr()),
          "pcadv_linear_bwd")
    return dx, dw, db


def adam_(param, grad, exp_avg, exp_avg_sq, step_count, lr, beta1, beta2, eps):
    """In-place torch.optim.Adam step on flat fp32 buffers; step_count is a
    device int32 tensor advanced by the call."""
    lib = _lib.load()
    n = param.numel()
    for t, nm in ((param, "param"), (grad, "grad"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq")):
        _req(t, nm)
        if t.numel() != n:
            raise ValueError(f"adam: {nm} has {t.numel()} elements, expected {n}")
    _req(step_count, "step_count", (1,), torch.int32)
    check(lib.pcadv_adam(ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), n, ptr(step_count),
                         lr, beta1, beta2, eps, stream_ptr()), "pcadv_adam")


# ---------------------------------------------------------------------------
# autograd
# ---------------------------------------------------------------------------

class PointFeatFunction(torch.autograd.Function):
    """PointNetfeat.forward (models/pointnet.py:109-132) as one fused pass:
    returns the global feature (C, 1024); the max-pool backward is sparse."""

    @staticmethod
    def forward(ctx, pts, w1, b1, w2, b2, w3, b3, w4, b4):
        gmax, gidx, x3 = feat_fwd(pts, w1, b1, w2, b2, w3, b3, w4, b4)
        ctx.save_for_backward(pts, w1, b1, w2, b2, w3, w4, x3, gidx)
        ctx.mark_non_differentiable(gidx)
        return gmax, gidx

    @staticmethod
    def backward(ctx, dgmax, _dgidx):
        pts, w1, b1, w2, b2, w3, w4, x3, gidx = ctx.saved_tensors
        g = feat_bwd(dgmax.contiguous(), gidx, pts, w1, b1, w2, b2, w3, w4, x3)
        return (None, *g)


class LinearFunction(torch.autograd.Function):
    """act(mask/(1-p) * (x w^T + b)) [+ I] for nn.Linear / 1x1 Conv1d layers."""

    @staticmethod
    def forward(ctx, x, w, b, act, mask, p, add_identity_k=0):
        y = linear_fwd(x, w, b, act, mask, p, add_identity_k)
        ctx.save_for_backward(x, w, y, mask if mask is not None else torch.empty(0))
        ctx.act, ctx.p, ctx.has_mask = act, p, mask is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y, mask = ctx.saved_tensors
        dx, dw, db = linear_bwd(dy.contiguous(), y, ctx.act, mask if ctx.has_mask else None, ctx.p,
                                x, w, need_dx=ctx.needs_input_grad[0],
                                need_dw=ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        return dx, dw, db, None, None, None, None


class PointwiseFunction(torch.autograd.Function):
    """1x1 Conv1d + activation over the points of point-major x (B, N, K)."""

    @staticmethod
    def forward(ctx, x, w, b, act):
        x = x.contiguous()
        y = pw_fwd(x, w, b, act)
        ctx.save_for_backward(x, w, y)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dy = dy.contiguous()
        act = ctx.act
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = pw_bwd_data(dy, y if act != ACT_NONE else None, act, _mat(w), x.shape[-1])
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            dwg, dbg = pw_bwd_weight(dy, y if act != ACT_NONE else None, act, x)
            dw, db = dwg.reshape(w.shape), dbg.reshape(-1)
        return dx, dw, db, None


class TransformFunction(torch.autograd.Function):
    """x (B, N, k) @ T (B, k, k): the feature transform (models/pointnet.py:120-121)."""

    @staticmethod
    def forward(ctx, x, T):
        x, T = x.contiguous(), T.contiguous()
        B, N, k = x.shape
        if T.shape != (B, k, k):
            raise ValueError(f"transform: expected T of shape {(B, k, k)}, got {tuple(T.shape)}")
        y = pw_fwd(x, T, None, ACT_NONE, kmajor=True, rows_per_w=N)
        ctx.save_for_backward(x, T)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, T = ctx.saved_tensors
        dy = dy.contiguous()
        N, k = x.shape[1], x.shape[2]
        dx = dT = None
        if ctx.needs_input_grad[0]:
            dx = pw_bwd_data(dy, None, ACT_NONE, T, k, kmajor=True, rows_per_w=N)
        if ctx.needs_input_grad[1]:
            dT, _ = pw_bwd_weight(dy, None, ACT_NONE, x, rows_per_group=N, kmajor=True,
                                  need_db=False)
        return dx, dT


class ConvMaxFunction(torch.autograd.Function):
    """1x1 Conv1d (128 -> O) then max over points, optionally with the ReLU before
    the max (T-Nets).  Returns the pooled (B, O); the backward is sparse."""

    @staticmethod
    def forward(ctx, x, w, b, relu_before_max):
        x = x.contiguous()
        gmax, gidx = conv_max_fwd(x, w, b, relu_before_max)
        ctx.save_for_backward(x, w, gmax, gidx)
        ctx.relu = bool(relu_before_max)
        return gmax

    @staticmethod
    def backward(ctx, dg):
        x, w, gmax, gidx = ctx.saved_tensors
        dx, dw, db = conv_max_bwd(dg.contiguous(), gidx, x, w, gmax if ctx.relu else None,
                                  need_dx=ctx.needs_input_grad[0])
        return dx, dw, db, None


class RegularizerFunction(torch.autograd.Function):
    """feature_transform_regularizer (models/pointnet.py:345-353)."""

    @staticmethod
    def forward(ctx, T):
        T = T.contiguous()
        reg, _ = tnet_reg_fwd(T)
        ctx.save_for_backward(T)
        return reg

    @staticmethod
    def backward(ctx, g):
        (T,) = ctx.saved_tensors
        return tnet_reg_bwd(T, g.to(torch.float32))
