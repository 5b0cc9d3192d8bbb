"""The fused feature-transform cls step (step.ClsFtTrainStep):
run_training_pointnet_cls's iteration (utils/trainer.py:254-268) with
PointNetCls(k=40, feature_transform=True) - CE + lambda_regu x
feature_transform_regularizer, backward, Adam - on the point-wise kernels and
the cls step's head (pcadv_cls_step part 3), against the numpy oracle
(oracle.cls_ft_forward_train / cls_ft_backward, pinned to the reference's own
g7 capture by tests/test_oracle_golden.py) and the reference's g7 step.

Gradients: against the oracle's backward on the device's own point-wise
activations and max-pool argmax (same-activation), per tensor 1e-4 of the
largest entry and 1e-5 relative L2.  Losses 1e-4.  Graph replay equals eager
bitwise.  MI355X only."""
import numpy as np
import pytest
import torch

from golden_util import check_tensor, check_tensor_rel, grad_err, load
from test_gpu_ft_step import _record

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _t(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, dtype)


def _model(seed):
    import adversarial_learning_on_pointclouds_amd as pc
    from oracle import pointnet_np as onp
    G = onp.make_params(onp.cls_ft_spec(40), seed=seed)
    m = pc.PointNetCls(k=40, feature_transform=True)
    m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in G.items()})
    return m.to(DEV), G


@pytest.mark.parametrize("B,N", [(4, 1024), (5, 384), (32, 1024)])
def test_cls_ft_step_vs_oracle_same_activation(monkeypatch, B, N):
    from adversarial_learning_on_pointclouds_amd.step import ClsFtTrainStep
    from oracle import pointnet_np as onp
    model, G = _model(61)
    st = ClsFtTrainStep(model, B, N, lambda_regu=0.001, seed=3)
    rng = np.random.default_rng(200 + B)
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    lab = rng.integers(0, 40, B)
    mask = (rng.random((B, 256)) >= 0.3).astype(np.float32)
    rec = _record(monkeypatch, "conv_max_fwd", lambda out: out[1])
    pw = _record(monkeypatch, "pw_fwd", lambda out: out)
    _record(monkeypatch, "pw_chain", lambda out: out, rec=pw, many=True)
    losses = st(_t(pts), _t(lab, torch.int64), mask=_t(mask), apply_adam=False).cpu().numpy()
    s3, c4 = (r.cpu().numpy() for r in rec[-2:])
    x1, x2, h1, h2, _, x3 = (a.cpu().numpy() for a in pw[-6:])
    acts = dict(x1=x1, x2=x2, h1=h1, h2=h2, x3=x3)
    # the oracle's own end to end step, for the printed distance and the losses
    l_own, r_own, g_own, aux = onp.cls_ft_step(G, pts, lab, mask, 1.0, 0.001)
    moved = [int((s3 != aux["am_stn"]).sum()), int((c4 != aux["am"]).sum())]
    print(f"B={B}: argmax the oracle's own forward moves (stn, conv4): {moved}")
    logits, cache = onp.cls_ft_forward_train(G, pts, mask, am_stn=s3, am=c4, acts=acts)
    l_ref, dce = onp.cross_entropy(logits, lab)
    reg = onp.feature_transform_regularizer(cache["trans"])
    grads = onp.cls_ft_backward(G, cache, dce, 0.001)
    assert abs(losses[0] - l_ref) < 1e-4 and abs(l_ref - l_own) < 1e-4
    assert abs(losses[1] - reg) < 1e-4 * max(1.0, abs(reg)) and abs(reg - r_own) < 1e-3
    assert np.abs(st.logits[:B].cpu().numpy() - logits).max() < 1e-4 * max(1.0, np.abs(logits).max())
    bad = []
    for nm, p in model.named_parameters():
        e = grad_err(p.grad.detach().cpu().numpy(), grads[nm])
        e2 = grad_err(p.grad.detach().cpu().numpy(), g_own[nm])
        print(f"{nm}: max {e[0]:.2e} l2 {e[1]:.2e} (end to end l2 {e2[1]:.2e})")
        if not (e[0] <= 1e-4 and e[1] <= 1e-5):
            bad.append((nm, e))
    assert not bad, bad


def test_cls_ft_step_golden_g7():
    """One run_training_pointnet_cls iteration with feature_transform=True
    against the reference's own capture g7 (loss, regulariser, every gradient
    per tensor at 1e-4 relative, every parameter after Adam at 1e-5)."""
    from adversarial_learning_on_pointclouds_amd.step import ClsFtTrainStep
    fx = load("g7_cls_ft_step.npz")
    model, _ = _model(int(fx["g_seed"]))
    pts = np.asarray(fx["pts"], np.float32)
    B, N = pts.shape[0], pts.shape[1]
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999))
    st = ClsFtTrainStep(model, B, N, optimizer=opt, lambda_cls=float(fx["lambda_cls"]),
                        lambda_regu=float(fx["lambda_regu"]))
    losses = st(_t(pts), _t(fx["labels"], torch.int64), mask=_t(fx["mask"])).cpu().numpy()
    assert abs(losses[0] - float(fx["loss_cls"])) < 1e-4
    assert abs(losses[1] - float(fx["reg"])) < 1e-3
    for name, p in model.named_parameters():
        check_tensor_rel(fx, "grad." + name, p.grad.detach().cpu().numpy(), tol=1e-4)
        check_tensor(fx, "param." + name, p.detach().cpu().numpy(), tol=1e-5)
    st.sync_optimizer_state()
    assert all(float(s["step"]) == 1 for s in opt.state.values())


def test_cls_ft_step_graph_replay_equals_eager():
    """Three iterations with device-drawn dropout and Adam: eager calls and
    replays of one captured graph leave bitwise the same parameters, moments,
    step count and losses."""
    from adversarial_learning_on_pointclouds_amd.step import ClsFtTrainStep
    B, N = 8, 512
    outs = []
    for graphed in (False, True):
        model, _ = _model(71)
        st = ClsFtTrainStep(model, B, N, seed=9)
        rng = np.random.default_rng(7)
        pts = _t(rng.uniform(-1, 1, (B, N, 3)))
        lab = _t(rng.integers(0, 40, B), torch.int64)
        g = st.capture_on(pts, lab) if graphed else None
        for k in range(3):
            r = np.random.default_rng(40 + k)
            pts.copy_(_t(r.uniform(-1, 1, (B, N, 3))))
            lab.copy_(_t(r.integers(0, 40, B), torch.int64))
            if graphed:
                g.replay()
            else:
                st(pts, lab)
        torch.cuda.synchronize()
        outs.append([t.clone() for t in (st.g_param, st.g_m, st.g_v, st.step_count, st.losses)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_cls_ft_trainer_uses_fused_step_and_matches_autograd(tmp_path, monkeypatch):
    """run_training_pointnet_cls over a DeviceCloudLoader with a
    feature_transform=True model runs the fused step (graphed); after 3
    iterations its parameters stay within 1e-3 of the parameters' movement of
    the autograd body (args.fused_ft = False, capturable Adam: the path before)
    on the same batches, dropout off; both log three loss lines."""
    import argparse
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import dataset as D, step as stepmod, trainer
    from oracle import pointnet_np as onp

    class _Log:
        def __init__(self):
            self.lines = []

        def info(self, s):
            self.lines.append(s)

    built = []
    orig = stepmod.ClsFtTrainStep.__init__

    def init(self, *a, **k):
        built.append(1)
        orig(self, *a, **k)
    monkeypatch.setattr(stepmod.ClsFtTrainStep, "__init__", init)
    rng = np.random.default_rng(81)
    data = rng.uniform(-1, 1, (8, 256, 3)).astype(np.float32)
    labels = rng.integers(0, 40, 8).astype(np.int32)
    G = onp.make_params(onp.cls_ft_spec(40), seed=82)
    res = []
    for fused_ft in (True, False):
        ds = D.ModelNetDatasetGT.__new__(D.ModelNetDatasetGT)
        ds.sample_list, ds.npoints, ds.data_augmentation = None, 256, False
        ds.select_data, ds.select_labels = data.copy(), labels.copy()
        ld = D.DeviceCloudLoader(ds, 4, seed=11, drop_last=True)
        m = pc.PointNetCls(k=40, feature_transform=True)
        m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in G.items()})
        m.dropout.p = 0.0
        m.cuda()
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, betas=(0.9, 0.999),
                               capturable=not fused_ft)
        args = argparse.Namespace(device="cuda", total_iterations=3, iter_save_epoch=10 ** 9,
                                  iter_test_epoch=10 ** 9, exp_dir=str(tmp_path), lambda_cls=1.0,
                                  lambda_regu=0.001, use_graph=True, fused_ft=fused_ft,
                                  batch_size=4)
        te = [(torch.from_numpy(data[:4].copy()), torch.from_numpy(labels[:4].astype(np.int64)))]
        log = _Log()
        trainer.run_training_pointnet_cls(ld, enumerate(ld), te, m, torch.nn.CrossEntropyLoss(),
                                          opt, log, log, None, args)
        res.append((torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu(),
                    [l for l in log.lines if l.startswith("iter")]))
    assert built == [1]  # the fused run built the step once, the autograd run none
    (pa, la), (pb, lb) = res
    p0 = torch.cat([torch.from_numpy(v).reshape(-1) for v in G.values()])
    # Adam moves every element by about lr whatever its gradient's size, so an
    # element whose gradient sits at rounding level can move either way in the
    # two paths: the movements are compared as vectors (relative L2)
    da, db = (pa - p0).double(), (pb - p0).double()
    rel = ((da - db).norm() / db.norm()).item()
    print(f"fused vs autograd parameter movement after 3 iterations: relative L2 {rel:.2e}, "
          f"max |diff| {(pa - pb).abs().max().item():.2e} of max movement {db.abs().max().item():.2e}")
    assert rel <= 1e-3
    assert len(la) == len(lb) == 3
