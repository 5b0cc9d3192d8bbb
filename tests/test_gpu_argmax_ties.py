"""k_conv4_max at three-way near-ties.

The kernel screens every point with three bf16 split products, keeps each
lane's top two, and re-evaluates the top two of every channel exactly; a third
point within the screening error of them is not re-checked (certifying it
measured +5.4 us per step, profiles/r06_argmax_cert_ab.txt).  These tests
force three points of a channel within 2^-20 of each other - below the
screening's resolution - and hold the documented guarantee: the pooled value
is the exact f32 dot product of the chosen point, the chosen point is one of
the three, and it lies within the screening bound of the true (f64) maximum,
2^-14 ||x_p|| ||w_o||.  An exact tie (three identical rows) must return the
first index, as torch.max does on CPU.  MI355X only."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(x3, w, b):
    from adversarial_learning_on_pointclouds_amd import ops
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    gmax, gidx = ops.conv4_max(t(x3), t(w), t(b))
    return gmax.cpu().numpy(), gidx.cpu().numpy()


def _tie_cloud(rng, C, N, o, eps, rows, exact=False):
    """x3 (C, N, 128) post-ReLU with, in every cloud, three rows `rows` whose
    channel-o values sit eps apart around a value above every other point's."""
    w = (rng.normal(size=(1024, 128)) / np.sqrt(128)).astype(np.float32)
    b = np.zeros(1024, np.float32)
    x3 = np.maximum(rng.normal(size=(C, N, 128)), 0).astype(np.float32) * 0.5
    wo = w[o].astype(np.float64)
    k = int(np.argmax(wo))  # the largest positive weight
    for c in range(C):
        v = x3[c].astype(np.float64) @ wo
        base = x3[c, int(np.argmax(v))].copy()
        base[k] += np.float32(0.25 / wo[k])  # lift the base row 0.25 above the rest
        for j, p in enumerate(rows):
            r = base.copy()
            if not exact:  # move the value by j * eps relative, in a low-weight coordinate
                kk = int(np.argmin(np.abs(wo) + (base <= 0) * 1e9))
                r[kk] = np.float32(r[kk] + j * eps * abs(base.astype(np.float64) @ wo) / max(abs(wo[kk]), 1e-3))
            x3[c, p] = r
    return x3, w, b


@pytest.mark.parametrize("order", [(100, 500, 900), (900, 500, 100), (5, 6, 7)])
def test_three_near_ties_within_the_screening_bound(order):
    rng = np.random.default_rng(sum(order))
    C, N, o = 8, 1024, 77
    x3, w, b = _tie_cloud(rng, C, N, o, 2.0 ** -20, order)
    gmax, gidx = _run(x3, w, b)
    for c in range(C):
        X = x3[c].astype(np.float64)
        Y = X @ w.T.astype(np.float64)
        p = int(gidx[c, o])
        assert p in order, (c, p, order)
        # the pooled value is the chosen point's exact f32 dot product
        assert abs(gmax[c, o] - Y[p, o]) <= 1e-6 * np.abs(X[p] * w[o]).sum() + 1e-30
        bound = 2.0 ** -14 * np.linalg.norm(X, axis=1).max() * np.linalg.norm(w[o])
        assert Y[:, o].max() - Y[p, o] <= bound, (Y[:, o].max() - Y[p, o], bound)


def test_three_exact_ties_take_the_first_index():
    rng = np.random.default_rng(3)
    C, N, o = 8, 1024, 301
    rows = (640, 130, 900)
    x3, w, b = _tie_cloud(rng, C, N, o, 0.0, rows, exact=True)
    _, gidx = _run(x3, w, b)
    assert (gidx[:, o] == min(rows)).all(), gidx[:, o]
