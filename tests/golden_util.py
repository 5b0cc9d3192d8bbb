"""Helpers to compare against the golden fixtures written by make_golden.py."""
import os

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return dict(np.load(os.path.join(HERE, name), allow_pickle=False))


def rel_err(a, ref):
    """max|a-ref| / max(1, max|ref|)  (SURVEY.md 8c tolerance form)."""
    a = np.asarray(a, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.max(np.abs(a - ref)) / max(1.0, float(np.max(np.abs(ref)))))


def grad_err(a, ref):
    """Per-tensor relative errors of a gradient: (max|a-ref| / max|ref|,
    ||a-ref||_2 / ||ref||_2).  Unlike rel_err there is no max(1, .) floor, so a
    zeroed or doubled gradient fails however small its entries are (at B=32 the
    conv gradients are ~1e-4, below rel_err's absolute 1e-3)."""
    a = np.asarray(a, np.float64).reshape(-1)
    r = np.asarray(ref, np.float64).reshape(-1)
    assert a.shape == r.shape, (a.shape, r.shape)
    d = a - r
    e_max = float(np.max(np.abs(d))) / max(float(np.max(np.abs(r))), 1e-30)
    e_l2 = float(np.linalg.norm(d)) / max(float(np.linalg.norm(r)), 1e-30)
    return e_max, e_l2


# Gradient tolerances (fp32 on both sides, different summation orders): the
# largest elementwise deviation within 1e-3 of the tensor's largest entry, and
# the relative L2 error within 1e-4.  A zeroed gradient has (1, 1), a doubled
# one (1, 1): both fail by three orders of magnitude.
GRAD_TOL_MAX = 1e-3
GRAD_TOL_L2 = 1e-4


def assert_grad_close(a, ref, name, tol_max=GRAD_TOL_MAX, tol_l2=GRAD_TOL_L2):
    e_max, e_l2 = grad_err(a, ref)
    assert e_max <= tol_max and e_l2 <= tol_l2, \
        f"{name}: max-rel {e_max:.3e} (tol {tol_max:g}), L2-rel {e_l2:.3e} (tol {tol_l2:g})"
    return e_max, e_l2


def adam_update_err(p_new, p_old, ref_new, ref_old, g_ref, g_floor=1e-5, rel_floor=1e-2):
    """Relative error of an Adam update: (p_new - p_old) against the oracle's
    (ref_new - ref_old), max over the elements whose reference gradient is
    above g_floor (1e3 x Adam's eps) and above rel_floor x the tensor's largest
    gradient (the gradient checks allow 1e-3 of that, so no selected element can
    change sign within them), relative to the largest reference update,
    each element's difference less one f32 spacing of its parameter (both sides
    round p_new to f32).  On those elements the first update is lr g / (|g| +
    eps) ~ lr sign(g): a wrong lr, bias correction or eps placement moves it by
    a large fraction, the rounding of the gradient does not."""
    p_old = np.asarray(p_old, np.float32).reshape(-1)
    du = np.asarray(p_new, np.float64).reshape(-1) - p_old.astype(np.float64)
    dr = np.asarray(ref_new, np.float64).reshape(-1) - np.asarray(ref_old, np.float64).reshape(-1)
    ga = np.abs(np.asarray(g_ref, np.float64).reshape(-1))
    sel = ga > max(g_floor, rel_floor * float(ga.max()))
    if not sel.any():
        return 0.0, 0
    d = np.maximum(np.abs(du - dr)[sel] - np.spacing(np.abs(p_old[sel])).astype(np.float64), 0.0)
    return float(d.max()) / max(float(np.abs(dr[sel]).max()), 1e-30), int(sel.sum())


def assert_adam_update_close(p_new, p_old, ref_new, ref_old, g_ref, name, tol=1e-3):
    e, n = adam_update_err(p_new, p_old, ref_new, ref_old, g_ref)
    assert n > 0, f"{name}: no gradient element above the floor: the check would be vacuous"
    assert e <= tol, f"{name}: Adam update rel err {e:.3e} over {n} elements (tol {tol:g})"
    return e


def check_tensor(fx, prefix, arr, tol=1e-3):
    """Compare a tensor against a fixture entry (full, or summary + samples)."""
    arr = np.asarray(arr, np.float32)
    if prefix in fx:
        ref = fx[prefix]
        assert arr.shape == ref.shape, (prefix, arr.shape, ref.shape)
        e = rel_err(arr, ref)
        assert e <= tol, f"{prefix}: rel err {e:.3e} > {tol}"
        return e
    flat = arr.reshape(-1).astype(np.float64)
    scale = max(1.0, float(fx[prefix + ".absmax"]))
    e_val = float(np.max(np.abs(flat[fx[prefix + ".idx"]] - fx[prefix + ".val"]))) / scale
    e_sum = abs(flat.sum() - float(fx[prefix + ".sum"])) / max(scale, abs(float(fx[prefix + ".sum"])))
    e_l2 = abs(np.sqrt((flat ** 2).sum()) - float(fx[prefix + ".l2"])) / max(1.0, float(fx[prefix + ".l2"]))
    e_max = abs(np.abs(flat).max() - float(fx[prefix + ".absmax"])) / scale
    e = max(e_val, e_l2, e_max)
    assert e <= tol, f"{prefix}: sample/l2/absmax err {e:.3e} > {tol}"
    assert e_sum <= max(tol, 1e-3), f"{prefix}: sum err {e_sum:.3e}"
    return e


def check_tensor_rel(fx, prefix, arr, tol=1e-3):
    """As check_tensor, but scaled by the tensor's own max|ref| (not max(1, .)):
    the strict form for gradients, which are far below 1."""
    arr = np.asarray(arr, np.float32)
    if prefix in fx:
        ref = np.asarray(fx[prefix], np.float64)
        assert arr.shape == ref.shape, (prefix, arr.shape, ref.shape)
        scale = max(float(np.max(np.abs(ref))), 1e-30)
        e = float(np.max(np.abs(arr.astype(np.float64) - ref))) / scale
        assert e <= tol, f"{prefix}: rel err {e:.3e} > {tol}"
        return e
    flat = arr.reshape(-1).astype(np.float64)
    scale = max(float(fx[prefix + ".absmax"]), 1e-30)
    e_val = float(np.max(np.abs(flat[fx[prefix + ".idx"]] - fx[prefix + ".val"]))) / scale
    e_l2 = abs(np.sqrt((flat ** 2).sum()) - float(fx[prefix + ".l2"])) / max(float(fx[prefix + ".l2"]), 1e-30)
    e_max = abs(np.abs(flat).max() - float(fx[prefix + ".absmax"])) / scale
    e = max(e_val, e_l2, e_max)
    assert e <= tol, f"{prefix}: sample/l2/absmax rel err {e:.3e} > {tol}"
    return e


def check_tensor_l2(fx, prefix, arr, tol=1e-2):
    """Relative L2 error ||a - ref|| / ||ref|| (full tensors), or of the l2 norm
    and the fixed-index samples (summarised ones): the form that tolerates the
    isolated ReLU-mask flips two f32 implementations of one network disagree on
    (a pre-activation within rounding of 0 routes a whole gradient element)."""
    a = np.asarray(arr, np.float64).reshape(-1)
    if prefix in fx:
        r = np.asarray(fx[prefix], np.float64).reshape(-1)
        e = float(np.linalg.norm(a - r) / max(np.linalg.norm(r), 1e-30))
    else:
        rv = np.asarray(fx[prefix + ".val"], np.float64)
        e_s = float(np.linalg.norm(a[fx[prefix + ".idx"]] - rv) / max(np.linalg.norm(rv), 1e-30))
        e_l2 = abs(np.linalg.norm(a) - float(fx[prefix + ".l2"])) / max(float(fx[prefix + ".l2"]), 1e-30)
        e = max(e_s, e_l2)
    assert e <= tol, f"{prefix}: relative L2 err {e:.3e} > {tol}"
    return e
