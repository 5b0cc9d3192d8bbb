"""PointNetSeg on the pcadv dense point-wise GEMM engine (csrc/gemm.hip).

Mirrors models/pointnet.py:261-317 of the reference: same class name,
constructor argument, forward signature (x: B x N x 3, cls: B x 1 x 16) and
return tuple (logits B x C x N, x_global B x 2048 x 1), same state_dict keys
and shapes, so reference checkpoints load unchanged.  The training loop
run_training_pointnet_seg (utils/trainer.py:310-400) is mirrored in
trainer.py.

Layout: activations are point-major rows (B*N rows).  conv1..conv5 write
their outputs straight into the column blocks of one [B*N][960] buffer, which
is both the next layer's input and the per-point part of fc1's 3024-wide
input (pointnet.py:304-306: [x1..x5 | tile(x_global) | tile(cls)]).  The
tiled parts are the same for every point of a cloud, so they are folded into
a per-cloud bias of fc1 (a B-row GEMM) instead of being materialised.
conv6 + ReLU + max over points never materialises the [B*N][2048] output: a
screened GEMM keeps per-tile candidates and the winner is re-evaluated in f32.

Numerics (precision="fp32", the default, the reference's dtype): every GEMM
multiplies the three-way bf16 splits of its f32 operands as six MFMA products
(hi hi, hi mid, mid hi, hi lo, mid mid, lo hi; f32 accumulate): f32-level
accuracy.  conv6's max is screened with three products and its winner (and
near-tie runner-up) re-evaluated as an exact f32 dot product, so the pooled
values are f32.  precision="bf16x3" (an explicitly labelled speed option,
below fp32): the forward and data-gradient GEMMs take three products of
hi / lo splits (relative error <= ~1.2e-5 of sum|a b| per layer), the forward
staged from bf16 planes its producers write.  Weight gradients (sums over all
B*N points, heavy cancellation) take six products in both modes.
tests/test_gpu_seg.py holds the tolerances.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn as nn

from . import _lib
from ._lib import check, stream_ptr
from .step import _step_tensor, set_optimizer_step

__all__ = ["PointNetSeg", "SegTrainStep", "seg_cross_entropy", "seg_forward", "seg_backward"]

_LOC = 960                       # x1..x5 widths 64 + 128 + 128 + 128 + 512
PRECISIONS = ("fp32", "bf16x3")
# bf16x3 mode: the forward's operands as bf16 hi / lo planes written once by
# their producers (pcadv_gemm_bf2; bitwise the f32-staged result);
# PCADV_SEG_PLANES=0 stages f32
_PLANES = os.environ.get("PCADV_SEG_PLANES", "1") == "1"
# fp32 mode: the forward GEMMs' weights as hi / mid / lo planes split once per
# step (pcadv_split_bf3 + pcadv_gemm_b3, bitwise the per-tile split).  Measured
# slower (seg 1.183 -> 1.200 ms, profiles/r06_seg_b3_ab.txt: the plane copies
# move 1.5x the f32 bytes per B tile, and the per-tile split they replace was
# hidden under the MFMAs), so off unless PCADV_SEG_B3=1
_B3 = os.environ.get("PCADV_SEG_B3", "0") == "1"


def _check_precision(precision):
    if precision not in PRECISIONS:
        raise ValueError(f"precision: one of {PRECISIONS}, got {precision!r}")
    return precision
_OFF = [0, 64, 192, 320, 448, 960]
_CONV = [(3, 64), (64, 128), (128, 128), (128, 128), (128, 512), (512, 2048)]


def _p(t, off=0):
    return ctypes.c_void_p(t.data_ptr() + 4 * off)


def _pb(t, off=0):  # bf16 tensors: element offsets of 2 bytes
    return ctypes.c_void_p(t.data_ptr() + 2 * off)


def _ws(nbytes, dev):
    return torch.empty(max(int(nbytes), 256), device=dev, dtype=torch.uint8)


class _Engine:
    """Thin, validated calls into the C ABI (every launch on the current stream)."""

    def __init__(self):
        self.lib = _lib.load()

    def gemm(self, a, lda, b, ldb, c, ldc, M, N, K, *, ta=0, tb=0, cmask=None, ldm=0, bias=None,
             bias_rows=None, rows_per_group=0, relu=False, accumulate=False, precise=False,
             a_off=0, b_off=0, c_off=0, m_off=0, cp=None, ldcp=0, cp_off=0):
        check(self.lib.pcadv_gemm(_p(a, a_off), lda, ta, _p(b, b_off), ldb, tb, _p(c, c_off), ldc,
                                  M, N, K, None if bias is None else _p(bias),
                                  None if bias_rows is None else _p(bias_rows), rows_per_group,
                                  int(relu), int(accumulate),
                                  None if cmask is None else _p(cmask, m_off), ldm, int(precise),
                                  None if cp is None else _pb(cp[0], cp_off),
                                  None if cp is None else _pb(cp[1], cp_off), ldcp, stream_ptr()),
              "pcadv_gemm")

    def gemm_bf2(self, ap, lda, bp, ldb, c, ldc, M, N, K, *, bias=None, bias_rows=None,
                 rows_per_group=0, relu=False, a_off=0, b_off=0, c_off=0, cp=None, ldcp=0,
                 cp_off=0):
        """A, B as (hi, lo) bf16 plane pairs; C f32 (+ its planes)."""
        check(self.lib.pcadv_gemm_bf2(_pb(ap[0], a_off), _pb(ap[1], a_off), lda, _pb(bp[0], b_off),
                                      _pb(bp[1], b_off), ldb, _p(c, c_off), ldc,
                                      None if cp is None else _pb(cp[0], cp_off),
                                      None if cp is None else _pb(cp[1], cp_off), ldcp, M, N, K,
                                      None if bias is None else _p(bias),
                                      None if bias_rows is None else _p(bias_rows),
                                      rows_per_group, int(relu), 0, None, 0, stream_ptr()),
              "pcadv_gemm_bf2")

    def gemm_b3(self, a, lda, bp, ldb, c, ldc, M, N, K, *, bias=None, bias_rows=None,
                rows_per_group=0, relu=False, a_off=0, c_off=0):
        """The six-product (fp32-mode) GEMM with B as its (hi, mid, lo) planes."""
        check(self.lib.pcadv_gemm_b3(_p(a, a_off), lda, _pb(bp[0]), _pb(bp[1]), _pb(bp[2]), ldb,
                                     _p(c, c_off), ldc, M, N, K,
                                     None if bias is None else _p(bias),
                                     None if bias_rows is None else _p(bias_rows), rows_per_group,
                                     int(relu), 0, stream_ptr()), "pcadv_gemm_b3")

    def split3(self, x, hi, mid, lo):
        """x f32 contiguous -> its hi, mid, lo bf16 planes (hi / mid = split's hi / lo)."""
        r, c = (1, x.numel()) if x.dim() == 1 else (x.shape[0], x.shape[1])
        check(self.lib.pcadv_split_bf3(_p(x), c, r, c, _pb(hi), _pb(mid), _pb(lo), c, stream_ptr()),
              "pcadv_split_bf3")

    def split(self, x, hi, lo):
        """x (rows, cols) f32 contiguous -> hi, lo bf16 of the same shape."""
        r, c = (1, x.numel()) if x.dim() == 1 else (x.shape[0], x.shape[1])
        check(self.lib.pcadv_split_bf2(_p(x), c, r, c, _pb(hi), _pb(lo), c, stream_ptr()),
              "pcadv_split_bf2")

    def gemm_desc(self, a, lda, b, ldb, c, ldc, M, N, K, *, ta=0, tb=0, cmask=None, ldm=0,
                  bias=None, bias_rows=None, rows_per_group=0, relu=False, accumulate=False,
                  precise=False, a_off=0, b_off=0, c_off=0, m_off=0):
        """pcadv_gemm's arguments as a pcadv_gemm_desc (for wgrad(..., pair=))."""
        return _lib.GemmDesc(_p(a, a_off), lda, ta, _p(b, b_off), ldb, tb, _p(c, c_off), ldc, M, N,
                             K, None if bias is None else _p(bias),
                             None if bias_rows is None else _p(bias_rows), rows_per_group,
                             int(relu), int(accumulate), None if cmask is None else _p(cmask, m_off),
                             ldm, int(precise), None, None, 0)

    def gemm_run(self, g):
        """Enqueue a pcadv_gemm_desc as its own launch."""
        check(self.lib.pcadv_gemm(g.a, g.lda, g.ta, g.b, g.ldb, g.tb, g.c, g.ldc, g.M, g.N, g.K,
                                  g.bias, g.bias_rows, g.rows_per_group, g.relu, g.accumulate,
                                  g.cmask, g.ldm, g.precise, g.c_hi, g.c_lo, g.ldcp, stream_ptr()),
              "pcadv_gemm")

    def wgrad(self, dz, ldz, x, ldx, rows, O, K, dw, ldo, *, db=None, gsum=None, rpg=0, dz_off=0,
              x_off=0, dw_off=0, fin=None, pair=None):
        """dw (+ db, gsum) = dz^T x over fixed-order slabs.

        fin: a caller-owned list; the finishing dw (and db) sums are then left to
        finish(fin), which runs all of them in one launch (the workspace rides in
        the list until then).  pair: a pcadv_gemm_desc (an independent data
        gradient) enqueued in the same launch as the slab GEMM.  Nothing is held
        by the library between calls: dropping `fin` abandons the sums."""
        nb = self.lib.pcadv_gemm_wgrad_workspace_bytes(rows, O, K, rpg)
        ws = _ws(nb, dz.device)
        if fin is None and pair is None:
            check(self.lib.pcadv_gemm_wgrad(
                _p(dz, dz_off), ldz, _p(x, x_off), ldx, rows, O, K, _p(dw, dw_off), ldo,
                None if db is None else _p(db), None if gsum is None else _p(gsum), rpg, 0, _p(ws),
                ws.numel(), stream_ptr()), "pcadv_gemm_wgrad")
            return
        d = _lib.WgradDesc(_p(dz, dz_off), ldz, _p(x, x_off), ldx, rows, O, K, _p(dw, dw_off), ldo,
                           None if db is None else _p(db), None if gsum is None else _p(gsum), rpg,
                           0, _p(ws), ws.numel())
        check(self.lib.pcadv_gemm_wgrad_slabs(ctypes.byref(d),
                                              None if pair is None else ctypes.byref(pair),
                                              stream_ptr()), "pcadv_gemm_wgrad_slabs")
        if fin is None:
            check(self.lib.pcadv_wgrad_finish(ctypes.byref(d), 1, stream_ptr()), "pcadv_wgrad_finish")
        else:
            fin.append((d, ws))

    def finish(self, fin):
        """Enqueue the finishing sums of the weight gradients collected in fin
        (one launch); the workspaces are released after it is enqueued (stream
        order keeps them until the launch has read them)."""
        if not fin:
            return
        arr = (_lib.WgradDesc * len(fin))(*[d for d, _ in fin])
        check(self.lib.pcadv_wgrad_finish(arr, len(fin), stream_ptr()), "pcadv_wgrad_finish")
        fin.clear()

    def wgrad_and_gemm(self, fin, wargs, wkw, g):
        """One layer's weight gradient (wgrad(*wargs, **wkw)) and its data gradient
        g (a pcadv_gemm_desc): one paired launch, or two (PCADV_GEMM_PAIR=0)."""
        if _PAIR:
            self.wgrad(*wargs, fin=fin, pair=g, **wkw)
        else:
            self.wgrad(*wargs, fin=fin, **wkw)
            self.gemm_run(g)

    def colsum(self, x, ld, M, N, out, *, ymask=None, ldm=0, x_off=0, m_off=0):
        nb = self.lib.pcadv_colsum_workspace_bytes(M, N)
        ws = _ws(nb, x.device)
        check(self.lib.pcadv_colsum(_p(x, x_off), None if ymask is None else _p(ymask, m_off), ld,
                                    ldm, M, N, _p(out), 0, _p(ws), ws.numel(), stream_ptr()),
              "pcadv_colsum")

    def group_colsum(self, x, ld, M, N, rows_per_group, out, *, ymask=None, ldm=0):
        check(self.lib.pcadv_group_colsum(_p(x), None if ymask is None else _p(ymask), ld, ldm, M,
                                          N, rows_per_group, _p(out), stream_ptr()),
              "pcadv_group_colsum")


_ENGINE = None


# weight gradients' finishing slab sums deferred and run in one launch at the
# end of the backward (PCADV_WGRAD_DEFER=0: one launch after each, for A/B runs)
_DEFER = os.environ.get("PCADV_WGRAD_DEFER", "1") != "0"
# each layer's weight and data gradients in one launch (_Engine.pair)
_PAIR = os.environ.get("PCADV_GEMM_PAIR", "1") != "0"
_SMALL = os.environ.get("PCADV_WGRAD_SMALL", "1") != "0"  # fc1's per-cloud columns: exact f32 kernel


def _engine():
    global _ENGINE
    if _ENGINE is None:
        _ENGINE = _Engine()
    return _ENGINE


def _wmat(w):
    return w.reshape(w.shape[0], -1)


def _check_dev(t, name, shape=None, dtype=torch.float32):
    if t.device.type != "cuda":
        raise ValueError(f"{name}: pcadv ops run on the HIP device only (got {t.device})")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")


def _weight_planes(W, Wf, wplanes=None):
    """(hi, lo) bf16 planes of conv2..conv6 and fc1..fc4, from ``wplanes`` (the
    caller's split of its flat parameter buffer: a list of 20 (hi, lo) pairs in
    state_dict order) or split here."""
    if wplanes is not None:
        return ([None] + [tuple(t.view(W[i].shape) for t in wplanes[2 * i]) for i in range(1, 6)],
                [tuple(t.view(Wf[i].shape) for t in wplanes[12 + 2 * i]) for i in range(4)])
    E = _engine()
    out = []
    for w in W[1:] + Wf:
        hi = torch.empty(w.shape, device=w.device, dtype=torch.bfloat16)
        lo = torch.empty_like(hi)
        E.split(w, hi, lo)
        out.append((hi, lo))
    return [None] + out[:5], out[5:]


def seg_forward(pts, cls, params, wplanes=None, precision="fp32", wplanes3=None):
    """PointNetSeg forward (pointnet.py:282-317) on the engine.  Returns a dict
    with logits (B*N, C) point-major, gmax (B, 2048), gidx (B, 2048) and every
    activation the backward needs.  Each layer's epilogue also writes its
    output's bf16 hi / lo planes, which the next layer's GEMM stages as they
    are (no per-tile splitting)."""
    E = _engine()
    B, N, _ = pts.shape
    M = B * N
    dev = pts.device
    pts = pts.contiguous()
    cvec = cls.reshape(B, -1).contiguous()
    W = [_wmat(params[2 * i]).contiguous() for i in range(6)]
    bc = [params[2 * i + 1].contiguous() for i in range(6)]
    Wf = [params[12 + 2 * i].contiguous() for i in range(4)]
    bf = [params[13 + 2 * i].contiguous() for i in range(4)]
    ncls = Wf[3].shape[0]
    fp32 = _check_precision(precision) == "fp32"
    planes = _PLANES and not fp32  # bf16x3: every forward GEMM staged from bf16 planes
    pf = fp32  # six-product forward GEMMs (staged from f32, split three ways per tile)
    # conv6's screen is three products in both modes (its winners are re-evaluated
    # in exact f32), staged from x5's planes: conv5's epilogue writes them
    c6p = _PLANES
    # fp32 mode with the caller's three-way weight planes (list of 20 (hi, mid,
    # lo) in state_dict order): the forward GEMMs stage B as plain copies
    b3 = fp32 and wplanes3 is not None
    if b3:
        W3p = [None] + [tuple(t.view(W[i].shape) for t in wplanes3[2 * i]) for i in range(1, 5)]
        Wf3p = [tuple(t.view(Wf[i].shape) for t in wplanes3[12 + 2 * i]) for i in range(4)]
    xloc = torch.empty(M, _LOC, device=dev)
    pl = lambda rows, cols: (torch.empty(rows, cols, device=dev, dtype=torch.bfloat16),  # noqa: E731
                             torch.empty(rows, cols, device=dev, dtype=torch.bfloat16))
    if c6p:
        Wp, Wfp = _weight_planes(W, Wf, wplanes)
    if planes:
        xp = pl(M, _LOC)
        x5p, x5ld, x5off = xp, _LOC, _OFF[4]
    elif c6p:
        x5p, x5ld, x5off = pl(M, 512), 512, 0
    # conv1..conv5 + ReLU into the column blocks of xloc
    E.gemm(pts, 3, W[0], 3, xloc, _LOC, M, 64, 3, bias=bc[0], relu=True, c_off=_OFF[0],
           precise=pf, cp=xp if planes else None, ldcp=_LOC, cp_off=_OFF[0])
    for i in range(1, 5):
        K, O = _CONV[i]
        if planes:
            E.gemm_bf2(xp, _LOC, Wp[i], K, xloc, _LOC, M, O, K, bias=bc[i], relu=True,
                       a_off=_OFF[i - 1], c_off=_OFF[i], cp=xp, ldcp=_LOC, cp_off=_OFF[i])
        elif b3 and not (i == 4 and c6p):
            E.gemm_b3(xloc, _LOC, W3p[i], K, xloc, _LOC, M, O, K, bias=bc[i], relu=True,
                      a_off=_OFF[i - 1], c_off=_OFF[i])
        else:
            last = i == 4 and c6p  # conv5 also writes x5's planes for conv6's screen
            E.gemm(xloc, _LOC, W[i], K, xloc, _LOC, M, O, K, bias=bc[i], relu=True,
                   a_off=_OFF[i - 1], c_off=_OFF[i], precise=pf, cp=x5p if last else None,
                   ldcp=x5ld if last else 0)
    # conv6 + ReLU + max over the points of each cloud
    gmax = torch.empty(B, 2048, device=dev)
    gidx = torch.empty(B, 2048, device=dev, dtype=torch.int32)
    nb = E.lib.pcadv_conv_max_x3_workspace_bytes(B, N, 2048)
    ws = _ws(nb, dev)
    if c6p:
        check(E.lib.pcadv_conv_max_bf2(_p(xloc, _OFF[4]), _LOC, _pb(x5p[0], x5off),
                                       _pb(x5p[1], x5off), x5ld, B, N, 512, _p(W[5]),
                                       _pb(Wp[5][0]), _pb(Wp[5][1]), _p(bc[5]), 2048, 1,
                                       _p(gmax), _p(gidx), _p(ws), ws.numel(), stream_ptr()),
              "pcadv_conv_max_bf2")
    else:
        check(E.lib.pcadv_conv_max_x3(_p(xloc, _OFF[4]), _LOC, B, N, 512, _p(W[5]), _p(bc[5]),
                                      2048, 1, _p(gmax), _p(gidx), _p(ws), ws.numel(),
                                      stream_ptr()), "pcadv_conv_max_x3")
    # fc1: per-cloud bias from the tiled global feature and class vector
    W1 = Wf[0]
    cb = torch.empty(B, 256, device=dev)
    E.gemm(gmax, 2048, W1, 3024, cb, 256, B, 256, 2048, bias=bf[0], b_off=960,
           precise=pf)
    E.gemm(cvec, cvec.shape[1], W1, 3024, cb, 256, B, 256, cvec.shape[1], b_off=3008,
           accumulate=True)
    h1 = torch.empty(M, 256, device=dev)
    h2 = torch.empty(M, 256, device=dev)
    h3 = torch.empty(M, 128, device=dev)
    logits = torch.empty(M, ncls, device=dev)
    if planes:
        h1p, h2p, h3p = pl(M, 256), pl(M, 256), pl(M, 128)
        E.gemm_bf2(xp, _LOC, Wfp[0], 3024, h1, 256, M, 256, _LOC, bias_rows=cb,
                   rows_per_group=N, relu=True, cp=h1p, ldcp=256)
        E.gemm_bf2(h1p, 256, Wfp[1], 256, h2, 256, M, 256, 256, bias=bf[1], relu=True, cp=h2p,
                   ldcp=256)
        E.gemm_bf2(h2p, 256, Wfp[2], 256, h3, 128, M, 128, 256, bias=bf[2], relu=True, cp=h3p,
                   ldcp=128)
        E.gemm_bf2(h3p, 128, Wfp[3], 128, logits, ncls, M, ncls, 128, bias=bf[3])
    elif b3:
        E.gemm_b3(xloc, _LOC, Wf3p[0], 3024, h1, 256, M, 256, _LOC, bias_rows=cb,
                  rows_per_group=N, relu=True)
        E.gemm_b3(h1, 256, Wf3p[1], 256, h2, 256, M, 256, 256, bias=bf[1], relu=True)
        E.gemm_b3(h2, 256, Wf3p[2], 256, h3, 128, M, 128, 256, bias=bf[2], relu=True)
        E.gemm_b3(h3, 128, Wf3p[3], 128, logits, ncls, M, ncls, 128, bias=bf[3])
    else:
        E.gemm(xloc, _LOC, W1, 3024, h1, 256, M, 256, _LOC, bias_rows=cb, rows_per_group=N,
               relu=True, precise=pf)
        E.gemm(h1, 256, Wf[1], 256, h2, 256, M, 256, 256, bias=bf[1], relu=True,
               precise=pf)
        E.gemm(h2, 256, Wf[2], 256, h3, 128, M, 128, 256, bias=bf[2], relu=True,
               precise=pf)
        E.gemm(h3, 128, Wf[3], 128, logits, ncls, M, ncls, 128, bias=bf[3], precise=pf)
    return dict(pts=pts, cvec=cvec, xloc=xloc, gmax=gmax, gidx=gidx, h1=h1, h2=h2, h3=h3, W=W,
                Wf=Wf, logits=logits, dims=(B, N, ncls), xp=xp if planes else None,
                precision=precision, x5p=(x5p, x5ld, x5off) if c6p else None,
                W6p=Wp[5] if c6p else None)


def seg_backward(fw, dlogits, dgmax_out=None, out=None):
    """Gradients of the 20 parameters (state_dict order) given dL/dlogits
    (B*N, C) (and optionally dL/dgmax), from the activations of seg_forward.
    `out`: optional list of 20 parameter-shaped tensors written in place."""
    E = _engine()
    pts, cvec, xloc, gmax, gidx = fw["pts"], fw["cvec"], fw["xloc"], fw["gmax"], fw["gidx"]
    h1, h2, h3, W, Wf = fw["h1"], fw["h2"], fw["h3"], fw["W"], fw["Wf"]
    B, N, ncls = fw["dims"]
    M = B * N
    dev = xloc.device
    pd = fw.get("precision", "fp32") == "fp32"  # six-product data gradients
    dl = torch.zeros(M, ncls, device=dev) if dlogits is None else dlogits.reshape(M, ncls).contiguous()
    # Every data-gradient GEMM applies the relu' of the layer below in its
    # epilogue (cmask), so each dz is stored masked once and read as is by the
    # weight gradient (which also forms the bias gradient) and the next GEMM.
    def _g(k, like):  # the k-th gradient (state_dict order): caller's buffer or a new one
        if out is not None:
            return out[k].view(like.shape) if hasattr(like, "shape") else out[k]
        return torch.empty_like(like) if hasattr(like, "shape") else torch.empty(like, device=dev)
    # the weight gradients' finishing slab sums wait in this local list and run
    # in one launch at the end (E.finish); an exception drops the list and
    # nothing is left behind (the library holds no state between calls)
    fin = [] if _DEFER else None
    # ---- fc4 .. fc2 -------------------------------------------------------
    dW4 = _g(18, Wf[3]); db4 = _g(19, ncls)
    dh3 = torch.empty(M, 128, device=dev)
    E.wgrad_and_gemm(fin, (dl, ncls, h3, 128, M, ncls, 128, dW4, 128), dict(db=db4),
                     E.gemm_desc(dl, ncls, Wf[3], 128, dh3, 128, M, 128, ncls, tb=1, cmask=h3,
                                 ldm=128, precise=pd))
    dW3 = _g(16, Wf[2]); db3 = _g(17, 128)
    dh2 = torch.empty(M, 256, device=dev)
    E.wgrad_and_gemm(fin, (dh3, 128, h2, 256, M, 128, 256, dW3, 256), dict(db=db3),
                     E.gemm_desc(dh3, 128, Wf[2], 256, dh2, 256, M, 256, 128, tb=1, cmask=h2,
                                 ldm=256, precise=pd))
    dW2 = _g(14, Wf[1]); db2 = _g(15, 256)
    dh1 = torch.empty(M, 256, device=dev)
    E.wgrad_and_gemm(fin, (dh2, 256, h1, 256, M, 256, 256, dW2, 256), dict(db=db2),
                     E.gemm_desc(dh2, 256, Wf[1], 256, dh1, 256, M, 256, 256, tb=1, cmask=h1,
                                 ldm=256, precise=pd))
    # ---- fc1: local columns (+ per-cloud sums s1), then the tiled columns --
    W1 = Wf[0]
    dW1 = _g(12, W1); db1 = _g(13, 256)
    s1 = torch.empty(B, 256, device=dev)  # per-cloud sums of dz1
    dloc = torch.empty(M, _LOC, device=dev)
    E.wgrad_and_gemm(fin, (dh1, 256, xloc, _LOC, M, 256, _LOC, dW1, 3024),
                     dict(db=db1, gsum=s1, rpg=N),
                     E.gemm_desc(dh1, 256, W1, 3024, dloc, _LOC, M, _LOC, 256, tb=1, cmask=xloc,
                                 ldm=_LOC, precise=pd))
    # the tiled global and class columns: B per-cloud rows, exact f32, one launch
    if not _SMALL:
        E.wgrad(s1, 256, gmax, 2048, B, 256, 2048, dW1, 3024, dw_off=960, fin=fin)
        E.wgrad(s1, 256, cvec, cvec.shape[1], B, 256, cvec.shape[1], dW1, 3024, dw_off=3008,
                fin=fin)
    else:
        check(E.lib.pcadv_wgrad_small(_p(s1), 256, B, 256, _p(gmax), 2048, 2048, _p(dW1, 960),
                                      _p(cvec), cvec.shape[1], cvec.shape[1], _p(dW1, 3008), 3024,
                                      0, stream_ptr()), "pcadv_wgrad_small")
    dg = torch.empty(B, 2048, device=dev)
    E.gemm(s1, 256, W1, 3024, dg, 2048, B, 2048, 256, tb=1, b_off=960, precise=pd)
    if dgmax_out is not None:
        dg += dgmax_out.reshape(B, 2048)
    # ---- conv6 + ReLU + max: the gradient reaches the argmax points -------
    dW6 = _g(10, W[5]); db6 = _g(11, 2048)
    check(E.lib.pcadv_conv_max_x3_bwd(_p(dg), _p(gmax), _p(gidx), _p(xloc, _OFF[4]), _LOC, B,
                                      N, 2048, 512, _p(W[5]), _p(dW6), _p(db6),
                                      _p(dloc, _OFF[4]), _LOC, 1, stream_ptr()),
          "pcadv_conv_max_x3_bwd")
    # ---- conv5 .. conv1 (each layer's output gradient also carries fc1's) --
    dWc = [None] * 6
    dbc = [None] * 6
    dWc[5], dbc[5] = dW6, db6
    for i in range(4, -1, -1):
        K, O = _CONV[i]
        dWc[i] = _g(2 * i, W[i])
        dbc[i] = _g(2 * i + 1, O)
        if i > 0:
            E.wgrad_and_gemm(fin, (dloc, _LOC, xloc, _LOC, M, O, K, dWc[i], K),
                             dict(db=dbc[i], dz_off=_OFF[i], x_off=_OFF[i - 1]),
                             E.gemm_desc(dloc, _LOC, W[i], K, dloc, _LOC, M, K, O, tb=1,
                                         cmask=xloc, ldm=_LOC, accumulate=True,
                                         precise=pd, a_off=_OFF[i],
                                         m_off=_OFF[i - 1], c_off=_OFF[i - 1]))
        else:
            E.wgrad(dloc, _LOC, pts, 3, M, O, K, dWc[i], K, db=dbc[i], dz_off=_OFF[i], fin=fin)
    # every weight gradient's slab sums (collected above) in one launch
    if fin is not None:
        E.finish(fin)
    grads = []
    for i in range(6):
        grads += [dWc[i].view(O_shape(i)), dbc[i]]
    grads += [dW1, db1, dW2, db2, dW3, db3, dW4, db4]
    return grads


class SegNetFunction(torch.autograd.Function):
    """PointNetSeg forward and its whole backward as one autograd node.

    Inputs: pts (B, N, 3), cls (B, 1, 16), then the 20 parameters in state_dict
    order.  Outputs: logits point-major (B, N, C), gmax (B, 2048), gidx (B, 2048)
    int32 (argmax over points, non-differentiable)."""

    @staticmethod
    def forward(ctx, precision, pts, cls, *params):
        fw = seg_forward(pts, cls, params, precision=precision)
        ctx.precision = precision
        ctx.save_for_backward(fw["pts"], fw["cvec"], fw["xloc"], fw["gmax"], fw["gidx"], fw["h1"],
                              fw["h2"], fw["h3"], *fw["W"], *fw["Wf"])
        ctx.dims = fw["dims"]
        ctx.mark_non_differentiable(fw["gidx"])
        B, N, ncls = fw["dims"]
        return fw["logits"].view(B, N, ncls), fw["gmax"], fw["gidx"]

    @staticmethod
    def backward(ctx, dlogits, dgmax_out, _dgidx):
        t = ctx.saved_tensors
        fw = dict(pts=t[0], cvec=t[1], xloc=t[2], gmax=t[3], gidx=t[4], h1=t[5], h2=t[6], h3=t[7],
                  W=list(t[8:14]), Wf=list(t[14:18]), dims=ctx.dims, precision=ctx.precision)
        B, N, ncls = ctx.dims
        dl = None if dlogits is None else dlogits.reshape(B * N, ncls)
        return (None, None, None, *seg_backward(fw, dl, dgmax_out))


def O_shape(i):
    K, O = _CONV[i]
    return (O, K, 1)


def seg_cross_entropy(logits_pm, seg, scale=1.0):
    """CrossEntropyLoss()(pred (B, C, N), seg (B, N)) for point-major logits
    (B, N, C): the mean over all points (pointnet/train_pointnet_seg.py:152,
    utils/trainer.py:344), on the device."""
    return _RowCE.apply(logits_pm, seg, float(scale))


class _RowCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits_pm, seg, scale):
        lib = _lib.load()
        B, N, C = logits_pm.shape
        M = B * N
        lg = logits_pm.reshape(M, C).contiguous()
        _check_dev(lg, "logits")
        lab = seg.reshape(M).to(torch.int64).contiguous()
        _check_dev(lab, "seg", dtype=torch.int64)
        loss = torch.empty((), device=lg.device)
        d = torch.empty_like(lg)
        ws = _ws(lib.pcadv_row_ce_workspace_bytes(M), lg.device)
        check(lib.pcadv_row_ce(_p(lg), C, _p(lab), M, C, 1.0, _p(loss), _p(d), _p(ws), ws.numel(),
                               stream_ptr()), "pcadv_row_ce")
        ctx.save_for_backward(d)
        ctx.shape = (B, N, C)
        return loss

    @staticmethod
    def backward(ctx, gl):
        (d,) = ctx.saved_tensors
        return (d * gl).view(ctx.shape), None, None


class PointNetSeg(nn.Module):
    """models/pointnet.py:261-317.  forward(x: B x N x 3, cls: B x 1 x 16) ->
    (logits B x NUM_SEG_CLASSES x N, x_global B x 2048 x 1)."""

    def __init__(self, NUM_SEG_CLASSES, *, precision="fp32"):
        super().__init__()
        self.output_dim = NUM_SEG_CLASSES
        # "fp32" (the reference's dtype) or "bf16x3" (labelled speed option)
        self.precision = _check_precision(precision)
        self.conv1 = nn.Conv1d(3, 64, 1)
        self.conv2 = nn.Conv1d(64, 128, 1)
        self.conv3 = nn.Conv1d(128, 128, 1)
        self.conv4 = nn.Conv1d(128, 128, 1)
        self.conv5 = nn.Conv1d(128, 512, 1)
        self.conv6 = nn.Conv1d(512, 2048, 1)
        self.fc1 = nn.Linear(3024, 256)
        self.fc2 = nn.Linear(256, 256)
        self.fc3 = nn.Linear(256, 128)
        self.fc4 = nn.Linear(128, self.output_dim)

    def forward_points(self, x, cls):
        """Point-major logits (B, N, C), x_global (B, 2048), argmax (B, 2048)."""
        B, N, c3 = x.shape
        if c3 != 3:
            raise ValueError(f"x: expected B x N x 3, got {tuple(x.shape)}")
        if cls.numel() != B * 16:
            raise ValueError(f"cls: expected B x 1 x 16, got {tuple(cls.shape)}")
        _check_dev(x, "x")
        params = [p for _, p in self.named_parameters()]
        return SegNetFunction.apply(self.precision, x.float().contiguous(),
                                    cls.float().reshape(B, 1, 16), *params)

    def forward(self, x, cls):
        logits, g, _ = self.forward_points(x, cls)
        return logits.permute(0, 2, 1), g.unsqueeze(2)


class SegTrainStep:
    """One iteration of run_training_pointnet_seg (utils/trainer.py:334-349:
    forward, CrossEntropyLoss over every point, (lambda_seg * l).backward(),
    optimizer.step() with Adam) as native launches on one stream, capturable
    into a HIP graph.

    The model's parameters become views of one flat f32 buffer, their .grad
    views of one flat gradient buffer (written in place by the backward), and
    the Adam moments are flat too (handed to a torch Adam's state as views, so
    optimizer.state_dict() stays meaningful); the update is one pcadv_adam
    launch over the whole network."""

    def __init__(self, model, optimizer=None, lr=1e-4, betas=(0.9, 0.999), eps=1e-8,
                 lambda_seg=1.0, device="cuda", keep_activations=False, precision=None):
        self.lib = _lib.load()
        # the model's precision unless given ("fp32" / "bf16x3")
        self.precision = _check_precision(precision or getattr(model, "precision", "fp32"))
        # keep_activations: hold the last step's forward tensors in self.fw (for
        # inspection / tests); off by default, so a step's per-point activations
        # (hundreds of MB at B=16, N=2048) are released when it returns
        self.keep_activations = bool(keep_activations)
        self.fw = None
        dev = torch.device(device)
        if dev.type != "cuda":
            raise ValueError("SegTrainStep runs on the HIP device only")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device, self.model = dev, model
        if optimizer is not None:
            g = optimizer.param_groups[0]
            lr, betas, eps = g["lr"], tuple(g["betas"]), g["eps"]
        self.lr, self.betas, self.eps, self.lambda_seg = float(lr), betas, float(eps), float(lambda_seg)
        named = list(model.named_parameters())
        offs, n = [], 0
        for _, p in named:
            offs.append(n)
            n += (p.numel() + 63) // 64 * 64  # 256-B aligned views
        self.numel = n
        self.param = torch.zeros(n, device=dev)
        self.grad = torch.zeros(n, device=dev)
        self.m = torch.zeros(n, device=dev)
        self.v = torch.zeros(n, device=dev)
        self.grad_views = []
        t0 = 0
        for (name, p), o in zip(named, offs):
            k = p.numel()
            self.param[o:o + k].copy_(p.detach().reshape(-1))
            st = optimizer.state.get(p) if optimizer is not None else None
            if st and "exp_avg" in st:  # Adam state the optimizer already holds carries over
                self.m[o:o + k].copy_(st["exp_avg"].detach().reshape(-1))
                self.v[o:o + k].copy_(st["exp_avg_sq"].detach().reshape(-1))
                t0 = max(t0, int(float(st.get("step", 0))))
            p.data = self.param[o:o + k].view_as(p)
            gv = self.grad[o:o + k].view_as(p)
            p.grad = gv
            self.grad_views.append(gv)
        if optimizer is not None:
            for (name, p), o in zip(named, offs):
                k = p.numel()
                optimizer.state[p] = {"step": _step_tensor(optimizer, p, t0),
                                      "exp_avg": self.m[o:o + k].view_as(p),
                                      "exp_avg_sq": self.v[o:o + k].view_as(p)}
        self.step_count = torch.full((1,), t0, device=dev, dtype=torch.int32)
        self.params = [p for _, p in named]
        # bf16 hi / lo planes of all parameters: one split per step feeds every
        # forward GEMM's weight operand
        self.wph = torch.empty(n, device=dev, dtype=torch.bfloat16)
        self.wpl = torch.empty(n, device=dev, dtype=torch.bfloat16)
        self.wplanes = [(self.wph[o:o + p.numel()], self.wpl[o:o + p.numel()])
                        for (_, p), o in zip(named, offs)]
        # fp32 mode: the three-way split (hi, mid = wph, wpl, and lo), one launch
        # per step, for the forward GEMMs' weight operands
        self.wpl3 = torch.empty(n, device=dev, dtype=torch.bfloat16) if _B3 else None
        self.wplanes3 = ([(self.wph[o:o + p.numel()], self.wpl[o:o + p.numel()],
                           self.wpl3[o:o + p.numel()]) for (_, p), o in zip(named, offs)]
                         if _B3 else None)
        self.optimizer = optimizer
        self.loss = torch.zeros((), device=dev)
        self.graph = None

    def __call__(self, pts, cls, seg, apply_adam=True):
        B, N, _ = pts.shape
        _check_dev(pts, "pts")
        if seg.shape != (B, N) or seg.dtype != torch.int64 or not seg.is_contiguous():
            raise ValueError("seg: expected contiguous int64 (B, N)")
        wpl = wpl3 = None
        if _B3 and self.precision == "fp32":  # hi / mid / lo: conv6 reads hi / mid
            _engine().split3(self.param, self.wph, self.wpl, self.wpl3)
            wpl, wpl3 = (self.wplanes if _PLANES else None), self.wplanes3
        elif _PLANES:  # every weight's planes (fp32 mode reads conv6's only)
            _engine().split(self.param, self.wph, self.wpl)
            wpl = self.wplanes
        fw = seg_forward(pts, cls.float().reshape(B, 1, 16), self.params, wplanes=wpl,
                         precision=self.precision, wplanes3=wpl3)
        if self.keep_activations:
            self.fw = fw  # the last step's activations (logits, x_global, argmax, ...)
        M, ncls = B * N, fw["dims"][2]
        d = torch.empty(M, ncls, device=self.device)
        ws = _ws(self.lib.pcadv_row_ce_workspace_bytes(M), self.device)
        check(self.lib.pcadv_row_ce(_p(fw["logits"]), ncls, _p(seg), M, ncls, self.lambda_seg,
                                    _p(self.loss), _p(d), _p(ws), ws.numel(), stream_ptr()),
              "pcadv_row_ce")
        seg_backward(fw, d, None, out=self.grad_views)
        if apply_adam:
            self.adam()
        return self.loss

    def adam(self):
        check(self.lib.pcadv_adam(_p(self.param), _p(self.grad), _p(self.m), _p(self.v), self.numel,
                                  _p(self.step_count), self.lr, self.betas[0], self.betas[1],
                                  self.eps, stream_ptr()), "pcadv_adam")

    def capture_on(self, pts, cls, seg):
        """A HIP graph of one step reading the given resident buffers (state is
        restored to what it was before the warm-up)."""
        saved = [t.clone() for t in (self.param, self.m, self.v, self.step_count)]
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self(pts, cls, seg)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self(pts, cls, seg)
        torch.cuda.synchronize()
        for dst, src in zip((self.param, self.m, self.v, self.step_count), saved):
            dst.copy_(src)
        return g

    @property
    def losses(self):
        """The loss as a 1-vector (the trainers' loss-ring interface)."""
        return self.loss.view(1)

    def graph_state(self):
        """What a captured iteration's warm-up changes (restored after it)."""
        return [self.param, self.m, self.v, self.step_count]

    def sync_hyper(self):
        """lr / betas / eps as the optimizer holds them now (a graph captured
        before keeps the old values: the trainer recaptures on a change)."""
        if self.optimizer is not None:
            g = self.optimizer.param_groups[0]
            self.lr, self.betas, self.eps = float(g["lr"]), tuple(float(b) for b in g["betas"]), \
                float(g["eps"])

    def sync_optimizer_state(self):
        if self.optimizer is not None:
            set_optimizer_step(self.optimizer, float(self.step_count.item()))
