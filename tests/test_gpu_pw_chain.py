"""pcadv_pw_chain (ops.pw_chain): consecutive point-wise layers of the
feature-transform extractor (models/pointnet.py:115-122 conv1, conv2, the
transform x2 T, conv3; :57-60 STNkd conv1, conv2) in one launch.  Every
layer's output must be BITWISE what the per-layer pcadv_pw_fwd launches write
(same fma chain / MFMA chain, bias and activation per layer), and those are
held to the oracle elsewhere (tests/test_gpu_tnet.py).  Shapes: full tiles,
ragged row counts, fewer tiles than the persistent grid, more tiles than two
rounds of it, and one transform per cloud.  MI355X only."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _w(rng, o, k, scale=0.3):
    return (torch.from_numpy(rng.standard_normal((o, k, 1)).astype(np.float32)) * scale).to(DEV)


def _b(rng, o):
    return torch.from_numpy(rng.standard_normal(o).astype(np.float32) * 0.1).to(DEV)


@pytest.mark.parametrize("C,N", [(64, 1024), (3, 333), (1, 64), (5, 130), (80, 1024)])
def test_chain_a_bitwise_per_layer(C, N):
    from adversarial_learning_on_pointclouds_amd import ops
    from adversarial_learning_on_pointclouds_amd.ops import ACT_RELU as RELU
    rng = np.random.default_rng(C * 7919 + N)
    pts = torch.from_numpy(rng.uniform(-1, 1, (C, N, 3)).astype(np.float32)).to(DEV)
    ws = [(_w(rng, 64, 3), _b(rng, 64)), (_w(rng, 64, 64), _b(rng, 64)),
          (_w(rng, 64, 64), _b(rng, 64)), (_w(rng, 128, 64), _b(rng, 128))]
    outs = ops.pw_chain(pts, [(w, b, RELU, False, 0) for w, b in ws])
    ref, x = [], pts
    for w, b in ws:
        x = ops.pw_fwd(x, w, b, RELU)
        ref.append(x)
    torch.cuda.synchronize()
    assert [tuple(o.shape) for o in outs] == [(C, N, 64)] * 3 + [(C, N, 128)]
    for i, (o, r) in enumerate(zip(outs, ref)):
        assert torch.equal(o, r), f"layer {i}: max |diff| {(o - r).abs().max().item()}"


@pytest.mark.parametrize("C,N", [(64, 1024), (3, 128), (33, 256), (2, 64)])
def test_chain_b_transform_bitwise_per_layer(C, N):
    """x2 T with one [64][64] transform per cloud (kmajor, rows_per_w = N), then
    conv3 + ReLU: the per-cloud fragments are refetched for every tile."""
    from adversarial_learning_on_pointclouds_amd import ops
    from adversarial_learning_on_pointclouds_amd.ops import ACT_NONE as NONE, ACT_RELU as RELU
    rng = np.random.default_rng(C * 31 + N)
    x2 = torch.from_numpy(np.maximum(rng.standard_normal((C, N, 64)), 0).astype(np.float32)).to(DEV)
    T = torch.from_numpy((np.eye(64) + 0.2 * rng.standard_normal((C, 64, 64))).astype(np.float32)).to(DEV)
    w3, b3 = _w(rng, 128, 64), _b(rng, 128)
    x2t, x3 = ops.pw_chain(x2, [(T, None, NONE, True, N), (w3, b3, RELU, False, 0)])
    r2t = ops.pw_fwd(x2, T, None, NONE, kmajor=True, rows_per_w=N)
    r3 = ops.pw_fwd(r2t, w3, b3, RELU)
    torch.cuda.synchronize()
    assert torch.equal(x2t, r2t)
    assert torch.equal(x3, r3)
    # and the transform itself against fp64
    ref = torch.einsum("cnk,cko->cno", x2.double(), T.double())
    assert (x2t.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


def test_chain_rejects_uninstantiated_shapes():
    from adversarial_learning_on_pointclouds_amd import ops
    from adversarial_learning_on_pointclouds_amd._lib import PcadvError
    from adversarial_learning_on_pointclouds_amd.ops import ACT_RELU as RELU
    rng = np.random.default_rng(3)
    x = torch.zeros(2, 64, 64, device=DEV)
    with pytest.raises(PcadvError, match="not instantiated"):
        ops.pw_chain(x, [(_w(rng, 64, 64), None, RELU, False, 0)])
