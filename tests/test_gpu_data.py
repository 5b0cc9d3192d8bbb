"""Device batch assembly: pcadv_gather_clouds through
DeviceCloudLoader against the reference's item semantics.  MI355X only."""
import os

import numpy as np
import pytest
import torch

from adversarial_learning_on_pointclouds_amd import dataset as D

pytestmark = pytest.mark.gpu
H5 = os.path.join(os.path.dirname(__file__), "golden", "h5")
EXP = np.load(os.path.join(H5, "expected.npz"))


def _list(tmp_path, names):
    p = tmp_path / "files.txt"
    p.write_text("".join(os.path.join(H5, n) + "\n" for n in names))
    return str(p)


def test_gather_with_explicit_noise_is_bitwise_the_reference_jitter(tmp_path):
    """Given the same f64 normal draws the device jitter equals
    jitter_point_cloud (modelNetData.py:80-91) + astype(float32) bit for bit."""
    ds = D.ModelNetDatasetGT(_list(tmp_path, ["modelnet_gzip.h5"]), None, npoints=64)
    ld = D.DeviceCloudLoader(ds, batch_size=3, shuffle=False)
    idx = torch.tensor([4, 0, 2], device="cuda", dtype=torch.int64)
    z = np.random.default_rng(1).standard_normal((3, 64, 3))
    z[0, :4] = [[9, -9, 0.2]] * 4  # beyond the clip
    pts, lab = ld.gather(idx, noise=z)
    src = EXP["modelnet_gzip/data"]
    ref = (np.clip(0.01 * z, -0.05, 0.05) + src[[4, 0, 2]]).astype(np.float32)
    assert np.array_equal(pts.cpu().numpy(), ref)
    assert np.array_equal(lab.cpu().numpy(), EXP["modelnet_gzip/label"][[4, 0, 2], 0].astype(np.int64))


def test_device_jitter_statistics_and_fresh_draws(tmp_path):
    ds = D.ModelNetDatasetGT(_list(tmp_path, ["modelnet_gzip.h5"]), None, npoints=64)
    ld = D.DeviceCloudLoader(ds, batch_size=5, shuffle=False, seed=3)
    idx = torch.arange(5, device="cuda", dtype=torch.int64)
    a, _ = ld.gather(idx)
    b, _ = ld.gather(idx)
    src = torch.from_numpy(EXP["modelnet_gzip/data"]).cuda()
    ja, jb = (a - src).cpu().numpy(), (b - src).cpu().numpy()
    assert np.abs(ja).max() <= 0.05 + 1e-6 and not np.array_equal(ja, jb)
    # many draws: N(0, 0.01^2) clipped at 5 sigma
    big = D.DeviceCloudLoader(D.ModelNetDatasetGT(_list(tmp_path, ["modelnet_gzip.h5"] * 40), None,
                                                  npoints=64), batch_size=200, shuffle=False)
    j = (big.gather(torch.arange(200, device="cuda"))[0].cpu().numpy()
         - np.tile(EXP["modelnet_gzip/data"], (40, 1, 1)))
    assert abs(j.mean()) < 5e-4 and abs(j.std() - 0.01) < 5e-4


def test_loader_epoch_covers_split_once(tmp_path):
    lst = _list(tmp_path, ["modelnet_gzip.h5", "modelnet_contig.h5"])
    ds = D.ModelNetDatasetGT(lst, np.array([6, 0, 3, 7, 1]), npoints=32, data_augmentation=False)
    ld = D.DeviceCloudLoader(ds, batch_size=2, shuffle=True, seed=5)
    assert len(ld) == 3
    seen = []
    for pts, lab in ld:
        assert pts.shape[1:] == (32, 3) and pts.dtype == torch.float32 and lab.dtype == torch.int64
        for p, l in zip(pts.cpu().numpy(), lab.cpu().numpy()):
            k = [i for i in range(len(ds)) if np.array_equal(ds.select_data[i], p)]
            assert len(k) == 1 and ds.select_labels[k[0]] == l
            seen.append(k[0])
    assert sorted(seen) == list(range(len(ds)))
    ng = D.DeviceCloudLoader(D.ModelNetDataset_noGT(lst, np.array([6, 0, 3, 7, 1]), npoints=32,
                                                    data_augmentation=False), 4, shuffle=False)
    first = next(iter(ng))
    assert isinstance(first, torch.Tensor) and first.shape == (3, 32, 3)


def test_shapenet_batches_with_part_ids(tmp_path):
    lst = _list(tmp_path, ["shapenet_latest.h5"])
    ds = D.ShapeNetDatasetGT(None, lst, num_classes=16, num_pts=50)
    ld = D.DeviceCloudLoader(ds, batch_size=4, shuffle=False)
    pts, oh, seg = ld.gather(torch.tensor([6, 2, 0, 5], device="cuda"))
    rows = [6, 2, 0, 5]
    assert np.array_equal(pts.cpu().numpy(), EXP["shapenet_latest/data"][rows])
    assert np.array_equal(seg.cpu().numpy(), EXP["shapenet_latest/pid"][rows].astype(np.int64))
    assert oh.shape == (4, 1, 16)
    assert np.array_equal(oh.cpu().numpy()[:, 0].argmax(1), EXP["shapenet_latest/label"][rows, 0])


def test_gather_multi_is_bitwise_the_single_gathers(tmp_path):
    """dataset.gather_at_multi (pcadv_gather_clouds_multi, one launch) writes
    exactly what each loader's gather_at writes: a labelled GT split with
    device jitter, a no-GT split of another batch size, and a ShapeNet split
    with part ids (different point counts per job)."""
    lst = _list(tmp_path, ["modelnet_gzip.h5", "modelnet_contig.h5"])
    rows = np.array([6, 0, 3, 7, 1])
    gt = D.DeviceCloudLoader(D.ModelNetDatasetGT(lst, rows, npoints=32), 3, seed=3)
    ng = D.DeviceCloudLoader(D.ModelNetDataset_noGT(lst, rows, npoints=24), 2, seed=4)
    sn = D.DeviceCloudLoader(D.ShapeNetDatasetGT(None, _list(tmp_path, ["shapenet_latest.h5"]),
                                                 num_classes=16, num_pts=50), 2, seed=5)
    dev = torch.device("cuda")
    jobs = []
    for ld in (gt, ng, sn):
        order = ld.epoch_order().to(dev)
        cursor = torch.zeros(1, dtype=torch.int32, device=dev)  # batch 0: in every order
        lab = (torch.zeros(ld.B, int(ld.labels.shape[1]), dtype=torch.int64, device=dev)
               if ld.labels is not None else None)
        seg = torch.zeros(ld.B, ld.npts, dtype=torch.int64, device=dev) if ld.segs is not None else None
        jobs.append((ld, order, cursor, torch.zeros(ld.B, ld.npts, 3, device=dev), lab, seg))
    D.gather_at_multi(jobs)
    multi = [[t.clone() for t in j[3:] if t is not None] for j in jobs]
    for ld, order, cursor, out, lab, seg in jobs:
        for t in (out, lab, seg):
            if t is not None:
                t.fill_(-7)
        ld.gather_at(order, cursor, out, lab, seg)
    for j, m in zip(jobs, multi):
        single = [t for t in j[3:] if t is not None]
        assert all(torch.equal(a, b) for a, b in zip(single, m))
    assert not torch.equal(multi[0][0], torch.zeros_like(multi[0][0]))


@pytest.mark.parametrize("kind", ["adv", "cls"])
def test_folded_epilogue_equals_the_epilogue_launch(kind):
    """The iteration epilogue run inside the step's finishing launch
    (pcadv_adv_args.epi_*, step.folded_epilogue) against the step followed by
    pcadv_iter_epilogue: same losses, parameters, loss-ring rows, ring count
    and counters, over three iterations."""
    from adversarial_learning_on_pointclouds_amd import trainer
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep, ClsTrainStep
    import adversarial_learning_on_pointclouds_amd as pc
    dev = torch.device("cuda")
    B, N = 8, 256
    g = torch.Generator().manual_seed(9)
    pg, pn = (torch.rand(B, N, 3, generator=g) * 2 - 1).to(dev), (torch.rand(B, N, 3, generator=g) * 2 - 1).to(dev)
    lab = torch.randint(0, 40, (B,), generator=g).to(dev)
    out = []
    for fold in (False, True):
        torch.manual_seed(0)
        model = pc.PointNetCls(k=40).to(dev)
        if kind == "adv":
            step = AdvTrainStep(model, pc.DeepConvDiscNet(40, 1).to(dev), B, N, seed=5, device=dev)
            call = lambda: step(pg, lab, pn)  # noqa: E731
        else:
            step = ClsTrainStep(model, B, N, seed=5, device=dev)
            call = lambda: step(pg, lab)  # noqa: E731
        ring = trainer._LossRing(lambda *a: None, 4 if kind == "adv" else 1, dev, slots=8)
        counters = torch.arange(4, dtype=torch.int32, device=dev)
        losses = step.losses if kind == "adv" else step.losses.view(-1)
        for it in range(3):
            if fold:
                with step.folded_epilogue(counters, 4, ring):
                    call()
            else:
                call()
                ring.write(losses, counters, 4)
        out.append([losses.clone(), ring.ring.clone(), ring.count.clone(), counters.clone(),
                    step.g_param.clone()])
    assert int(out[1][2]) == 3 and out[1][3].tolist() == [3, 4, 5, 6]
    for a, b in zip(*out):
        assert torch.equal(a, b)


@pytest.mark.parametrize("kind", ["adv", "cls"])
def test_folded_gather_equals_the_gather_launch(kind):
    """The step gathering its own input batches in its first launch
    (pcadv_adv_args.gather, step.folded_gather) against gather_at + the step:
    the same jittered points and labels in the input buffers, the same losses
    and parameters (three iterations, the loaders' RNG steps and cursors
    advanced between them)."""
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep, ClsTrainStep
    import adversarial_learning_on_pointclouds_amd as pc
    dev = torch.device("cuda")
    B, N = 4, 96
    rng = np.random.default_rng(77)

    def mem(cls, n):
        ds = cls.__new__(cls)
        ds.sample_list, ds.npoints, ds.data_augmentation = None, N, True
        ds.select_data = rng.uniform(-1, 1, (n, N, 3)).astype(np.float32)
        if cls is D.ModelNetDatasetGT:
            ds.select_labels = rng.integers(0, 40, n).astype(np.int32)
        return ds
    gds, nds = mem(D.ModelNetDatasetGT, 12), mem(D.ModelNetDataset_noGT, 12)
    out = []
    for fold in (False, True):
        gt = D.DeviceCloudLoader(gds, B, seed=21)
        ng = D.DeviceCloudLoader(nds, B, seed=22)
        lds = (gt, ng) if kind == "adv" else (gt,)
        orders = [ld.epoch_order().to(dev) for ld in lds]
        cursors = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in lds]
        pts = [torch.zeros(B, N, 3, device=dev) for _ in lds]
        lab = torch.zeros(B, 1, dtype=torch.int64, device=dev)
        torch.manual_seed(0)
        model = pc.PointNetCls(k=40).to(dev)
        if kind == "adv":
            step = AdvTrainStep(model, pc.DeepConvDiscNet(40, 1).to(dev), B, N, seed=3, device=dev)
            call = lambda: step(pts[0], lab[:, 0], pts[1])  # noqa: E731
        else:
            step = ClsTrainStep(model, B, N, seed=3, device=dev)
            call = lambda: step(pts[0], lab[:, 0])  # noqa: E731
        rec = []
        for it in range(3):
            labs = [lab] + [None] * (len(lds) - 1)
            if fold:
                jobs = [ld._gather_job(o, c, p, l)
                        for ld, o, c, p, l in zip(lds, orders, cursors, pts, labs)]
                with step.folded_gather(jobs):
                    call()
            else:
                for ld, o, c, p, l in zip(lds, orders, cursors, pts, labs):
                    ld.gather_at(o, c, p, l)
                call()
            rec += [t.clone() for t in pts] + [lab.clone(), step.losses.clone()]
            for ld, c in zip(lds, cursors):
                ld.step += 1
                c += 1
        rec.append(step.g_param.clone())
        out.append(rec)
    for i, (a, b) in enumerate(zip(*out)):
        assert torch.equal(a, b), i
    assert not torch.equal(out[0][0], out[0][len(out[0]) // 3])  # fresh batches per iteration
    # the labels the step reads must be the ones job 0 gathers
    other = torch.zeros_like(lab)
    jobs = [ld._gather_job(o, c, p, l) for ld, o, c, p, l in
            zip(lds, orders, cursors, pts, [other] + [None] * (len(lds) - 1))]
    with pytest.raises(Exception, match="gathered labels"):
        with step.folded_gather(jobs):
            call()


class _Log:
    def __init__(self):
        self.lines = []

    def info(self, s):
        self.lines.append(s)


def test_seg_trainer_end_to_end_on_device_batches(tmp_path):
    """run_training_pointnet_seg (trainer.py:310-400) fed by DeviceCloudLoader
    over a ShapeNet-format file: fused SegTrainStep iterations, run_testing_seg
    (accuracy + IoU), checkpoints."""
    import argparse
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import trainer
    torch.manual_seed(0)
    lst = _list(tmp_path, ["shapenet_latest.h5"])
    train = D.ShapeNetDatasetGT(np.arange(5), lst, num_classes=16, num_pts=48)
    test = D.ShapeNetDatasetGT(None, lst, num_classes=16, num_pts=48)
    tl = D.DeviceCloudLoader(train, batch_size=2, shuffle=True, seed=1, drop_last=True)
    vl = D.DeviceCloudLoader(test, batch_size=3, shuffle=False)
    model = pc.PointNetSeg(50).cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    args = argparse.Namespace(device="cuda", total_iterations=6, iter_save_epoch=4,
                              iter_test_epoch=5, exp_dir=str(tmp_path), tensorboard=False,
                              lambda_seg=1.0, input_pts=48)
    log = _Log()
    accu, cat_iou, all_iou = trainer.run_training_pointnet_seg(
        tl, enumerate(tl), vl, test, model, torch.nn.CrossEntropyLoss(), opt, log, log, None, args)
    losses = [float(l.split("loss_seg = ")[1]) for l in log.lines if "loss_seg" in l]
    assert len(losses) == 6 and all(np.isfinite(losses)) and losses[-1] < losses[0]
    # the fixture holds few object categories: the category mean is NaN (the
    # reference's np.mean over empty lists, too), so its maximum stays -inf
    assert 0.0 <= all_iou <= 1.0 and accu >= 0.0 and (cat_iou == float("-inf") or 0 <= cat_iou <= 1)
    assert (tmp_path / "model_train_epoch_0.pth").exists()


def _seg_run(tmp_path, use_graph, drop_last, iters=7):
    import argparse
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import trainer
    torch.manual_seed(0)
    lst = _list(tmp_path, ["shapenet_latest.h5"])
    train = D.ShapeNetDatasetGT(np.arange(5), lst, num_classes=16, num_pts=48)
    test = D.ShapeNetDatasetGT(None, lst, num_classes=16, num_pts=48)
    tl = D.DeviceCloudLoader(train, batch_size=2, shuffle=True, seed=1, drop_last=drop_last)
    vl = D.DeviceCloudLoader(test, batch_size=3, shuffle=False)
    model = pc.PointNetSeg(50).cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    args = argparse.Namespace(device="cuda", total_iterations=iters, iter_save_epoch=10 ** 9,
                              iter_test_epoch=4, exp_dir=str(tmp_path), tensorboard=False,
                              lambda_seg=1.0, input_pts=48, use_graph=use_graph)
    log = _Log()
    graphs = []
    orig = trainer._SegGraphedIteration.replay

    def spy(self, semi=False):
        graphs.append(1)
        return orig(self, semi)
    trainer._SegGraphedIteration.replay = spy
    try:
        trainer.run_training_pointnet_seg(tl, enumerate(tl), vl, test, model,
                                          torch.nn.CrossEntropyLoss(), opt, log, log, None, args)
    finally:
        trainer._SegGraphedIteration.replay = orig
    params = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu()
    return params, [l for l in log.lines if "loss_seg" in l], len(graphs), opt


@pytest.mark.parametrize("drop_last", [True, False])
def test_graphed_seg_trainer_equals_eager(tmp_path, drop_last):
    """run_training_pointnet_seg over a ShapeNet DeviceCloudLoader with each
    full iteration (gather + one-hot + SegTrainStep + epilogue) replayed as one
    HIP graph, loss lines read from the device ring: bitwise the eager loop
    (parameters, loss lines, Adam step count), across epoch wrap-arounds and,
    with drop_last=False, the ragged last batch (run eagerly in between)."""
    pa, la, na, opt = _seg_run(tmp_path, True, drop_last)
    pb, lb, nb, _ = _seg_run(tmp_path, False, drop_last)
    assert na == (7 if drop_last else 5) and nb == 0
    assert torch.equal(pa, pb)
    assert la == lb and len(la) == 7
    assert all(float(st["step"]) == 7 for st in opt.state.values())


def test_semi_trainer_end_to_end_on_device_batches(tmp_path):
    """run_training_semi (trainer.py:611-847) fed by DeviceCloudLoader over
    ModelNet-format files with the GT / no-GT split of sample_list."""
    import argparse
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import trainer
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    torch.manual_seed(0)
    lst = _list(tmp_path, ["modelnet_gzip.h5", "modelnet_contig.h5"])
    gt_rows = np.array([0, 2, 5, 7])
    gt = D.DeviceCloudLoader(D.ModelNetDatasetGT(lst, gt_rows, npoints=32), 2, drop_last=True)
    ng = D.DeviceCloudLoader(D.ModelNetDataset_noGT(lst, gt_rows, npoints=32), 2, drop_last=True)
    te = D.DeviceCloudLoader(D.ModelNetDatasetGT(lst, None, npoints=32, data_augmentation=False), 2)
    model, model_D = pc.PointNetCls(k=40).cuda(), pc.DeepConvDiscNet(40, 1).cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999))
    opt_D = torch.optim.Adam(model_D.parameters(), lr=1e-4, betas=(0.9, 0.999))
    args = argparse.Namespace(device="cuda", total_iterations=5, iter_save_epoch=10 ** 9,
                              iter_test_epoch=10 ** 9, exp_dir=str(tmp_path), tensorboard=False,
                              lambda_cls=1.0, lambda_adv=0.001, lambda_semi=1.0, semi_start=2,
                              semi_TH=-1e9, batch_size=2)
    log = _Log()
    trainer.run_training_semi(gt, ng, enumerate(gt), enumerate(ng), te, model, model_D,
                              torch.nn.BCEWithLogitsLoss(), torch.nn.CrossEntropyLoss(),
                              torch.nn.CrossEntropyLoss(ignore_index=255), opt, opt_D,
                              ImagePool(0), ImagePool(0), log, log, None, args)
    lines = [l for l in log.lines if l.startswith("iter")]
    assert len(lines) == 5
    for p in list(model.parameters()) + list(model_D.parameters()):
        assert torch.isfinite(p).all()


def test_run_training_uneven_batches_keeps_adam_state():
    """run_training (trainer.py:403-608) with drop_last=False loaders whose
    GT / no-GT batch sizes differ on some iterations: those run the autograd
    path with the torch optimizers, the rest the fused step.  The Adam state
    (moments, bias-correction step count) must carry across both, so the
    generator's parameter trajectory equals the oracle's five Adam steps.
    lambda_adv = 0 and dropout p = 0 make G's trajectory independent of the
    random soft D labels and masks."""
    import argparse
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import trainer
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    from oracle import pointnet_np as onp
    N = 256
    G = onp.make_params(onp.cls_spec(40), seed=12)
    Dp = onp.make_params(onp.disc_spec(40, 1), seed=13, init="xavier")
    rng = np.random.default_rng(14)
    mk = lambda b: rng.uniform(-1, 1, (b, N, 3)).astype(np.float32)
    gt = [(mk(4), rng.integers(0, 40, 4)), (mk(3), rng.integers(0, 40, 3))]
    ng = [mk(4), mk(4), mk(2)]
    model = pc.PointNetCls(k=40)
    model.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in G.items()})
    model.dropout.p = 0.0
    model_D = pc.DeepConvDiscNet(40, 1)
    model_D.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in Dp.items()})
    model.cuda()
    model_D.cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999))
    opt_D = torch.optim.Adam(model_D.parameters(), lr=1e-4, betas=(0.9, 0.999))
    tgt = [(torch.from_numpy(p), torch.from_numpy(l)) for p, l in gt]
    tng = [torch.from_numpy(p) for p in ng]
    iters = 5
    args = argparse.Namespace(device="cuda", total_iterations=iters, iter_save_epoch=10 ** 9,
                              iter_test_epoch=10 ** 9, exp_dir="/tmp", tensorboard=False,
                              lambda_cls=1.0, lambda_adv=0.0, batch_size=4)
    log = _Log()
    trainer.run_training(tgt, tng, enumerate(tgt), enumerate(tng), [tgt[0]], model, model_D,
                         torch.nn.BCEWithLogitsLoss(), torch.nn.CrossEntropyLoss(), opt, opt_D,
                         ImagePool(0), ImagePool(0), log, log, None, args)
    # the oracle over the same batch sequence (GT i % 2, no-GT i % 3)
    G0 = {k: v.copy() for k, v in G.items()}
    oG, oD = onp.Adam(G), onp.Adam(Dp)
    for i in range(iters):
        pg, lab = gt[i % 2]
        pn = ng[i % 3]
        # masks None: no dropout scale (p = 0)
        onp.adv_step(G, Dp, oG, oD, pg, lab, pn, None, None, np.full((len(pg), 1), 0.9, np.float32),
                     np.full((len(pn), 1), 0.1, np.float32), lambda_adv=0.0)
    for name, p in model.named_parameters():
        d_gpu = p.detach().cpu().numpy().astype(np.float64) - G0[name]
        d_ref = G[name].astype(np.float64) - G0[name]
        e = np.linalg.norm(d_gpu - d_ref) / max(np.linalg.norm(d_ref), 1e-30)
        assert e < 1e-2, (name, e)   # a stale bias correction moves these by ~0.5
    for st in opt.state.values():
        assert float(st["step"]) == iters
    assert all(p.grad is not None for p in model.parameters())


def test_loader_streams_independent_and_index_checked(tmp_path):
    """GT and no-GT loaders given the same seed draw different jitter fields
    (the dataset kind is part of the Philox key), default-seeded loaders
    differ too, and gather() rejects indices outside the split."""
    lst = _list(tmp_path, ["modelnet_gzip.h5", "modelnet_contig.h5"])
    rows = np.array([0, 2, 5, 7])
    gt_ds = D.ModelNetDatasetGT(lst, rows, npoints=32)
    ng_ds = D.ModelNetDataset_noGT(lst, rows, npoints=32)
    idx = torch.zeros(1, device="cuda", dtype=torch.int64)
    jit = []
    for ld in (D.DeviceCloudLoader(gt_ds, 1, seed=7), D.DeviceCloudLoader(ng_ds, 1, seed=7),
               D.DeviceCloudLoader(gt_ds, 1), D.DeviceCloudLoader(gt_ds, 1)):
        out = ld.gather(idx)
        pts = out[0] if isinstance(out, tuple) else out
        jit.append((pts.cpu().numpy() - ld.ds.select_data[0]))
    for a in range(4):
        for b in range(a + 1, 4):
            assert not np.allclose(jit[a], jit[b]), (a, b)
    ld = D.DeviceCloudLoader(gt_ds, 2, seed=1)
    with pytest.raises(IndexError):
        ld.gather(torch.tensor([0, len(gt_ds)], device="cuda"))
    with pytest.raises(IndexError):
        ld.gather(torch.tensor([-1], device="cuda"))


def test_run_training_step_rebuild_keeps_adam_step_count():
    """A larger batch mid-run rebuilds the fused step (trainer.py): the new step
    adopts the Adam moments AND the completed-step count of the old one, so the
    bias correction continues (utils/trainer.py:558-559 keeps one Adam state
    over the whole run).  GT / no-GT batches of 4, 4, 8 clouds (the 8 forces the
    rebuild at i_iter 2), lambda_adv = 0 and dropout p = 0: the generator's
    trajectory must equal the oracle's five Adam steps."""
    import argparse
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import trainer
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    from oracle import pointnet_np as onp
    N = 128
    G = onp.make_params(onp.cls_spec(40), seed=22)
    Dp = onp.make_params(onp.disc_spec(40, 1), seed=23, init="xavier")
    rng = np.random.default_rng(24)
    mk = lambda b: rng.uniform(-1, 1, (b, N, 3)).astype(np.float32)
    gt = [(mk(b), rng.integers(0, 40, b)) for b in (4, 4, 8)]
    ng = [mk(b) for b in (4, 4, 8)]
    model = pc.PointNetCls(k=40)
    model.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in G.items()})
    model.dropout.p = 0.0
    model_D = pc.DeepConvDiscNet(40, 1)
    model_D.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in Dp.items()})
    model.cuda()
    model_D.cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999))
    opt_D = torch.optim.Adam(model_D.parameters(), lr=1e-4, betas=(0.9, 0.999))
    tgt = [(torch.from_numpy(p), torch.from_numpy(l)) for p, l in gt]
    tng = [torch.from_numpy(p) for p in ng]
    iters = 5
    args = argparse.Namespace(device="cuda", total_iterations=iters, iter_save_epoch=10 ** 9,
                              iter_test_epoch=10 ** 9, exp_dir="/tmp", tensorboard=False,
                              lambda_cls=1.0, lambda_adv=0.0, batch_size=4)
    log = _Log()
    trainer.run_training(tgt, tng, enumerate(tgt), enumerate(tng), [tgt[0]], model, model_D,
                         torch.nn.BCEWithLogitsLoss(), torch.nn.CrossEntropyLoss(), opt, opt_D,
                         ImagePool(0), ImagePool(0), log, log, None, args)
    G0 = {k: v.copy() for k, v in G.items()}
    oG, oD = onp.Adam(G), onp.Adam(Dp)
    for i in range(iters):
        pg, lab = gt[i % 3]
        pn = ng[i % 3]
        onp.adv_step(G, Dp, oG, oD, pg, lab, pn, None, None, np.full((len(pg), 1), 0.9, np.float32),
                     np.full((len(pn), 1), 0.1, np.float32), lambda_adv=0.0)
    for name, p in model.named_parameters():
        d_gpu = p.detach().cpu().numpy().astype(np.float64) - G0[name]
        d_ref = G[name].astype(np.float64) - G0[name]
        e = np.linalg.norm(d_gpu - d_ref) / max(np.linalg.norm(d_ref), 1e-30)
        assert e < 1e-2, (name, e)   # a restarted bias correction moves these by ~0.3
    for st in opt.state.values():
        assert float(st["step"]) == iters


def _pool_run(pool_size, fused, iters=6, sizes=(4, 4, 4)):
    """run_training over host batches of 4 + 4 clouds with ImagePool(pool_size)
    on both D inputs; fused=False forces the reference's autograd body (a
    CrossEntropyLoss subclass is off the fused step's configuration)."""
    import argparse
    import random
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import trainer
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    from oracle import pointnet_np as onp

    class _CE(torch.nn.CrossEntropyLoss):
        pass

    N = 256
    G = onp.make_params(onp.cls_spec(40), seed=41)
    Dp = onp.make_params(onp.disc_spec(40, 1), seed=42, init="xavier")
    rng = np.random.default_rng(43)
    gt = [(torch.from_numpy(rng.uniform(-1, 1, (b, N, 3)).astype(np.float32)),
           torch.from_numpy(rng.integers(0, 40, b))) for b in sizes]
    ng = [torch.from_numpy(rng.uniform(-1, 1, (b, N, 3)).astype(np.float32)) for b in sizes]
    model, model_D = pc.PointNetCls(k=40), pc.DeepConvDiscNet(40, 1)
    model.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in G.items()})
    model_D.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in Dp.items()})
    model.dropout.p = 0.0  # no dropout draws: both bodies draw only D's soft labels from torch
    model.cuda()
    model_D.cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999))
    opt_D = torch.optim.Adam(model_D.parameters(), lr=1e-4, betas=(0.9, 0.999))
    args = argparse.Namespace(device="cuda", total_iterations=iters, iter_save_epoch=10 ** 9,
                              iter_test_epoch=10 ** 9, exp_dir="/tmp", tensorboard=False,
                              lambda_cls=1.0, lambda_adv=0.01, batch_size=4)
    pools = ImagePool(pool_size), ImagePool(pool_size)
    random.seed(5)
    torch.manual_seed(6)
    log = _Log()
    trainer.run_training(gt, ng, enumerate(gt), enumerate(ng), [gt[0]], model, model_D,
                         torch.nn.BCEWithLogitsLoss(), torch.nn.CrossEntropyLoss() if fused else _CE(),
                         opt, opt_D, *pools, log, log, None, args)
    lines = [l for l in log.lines if l.startswith("iter")]
    loss_d = np.array([float(l.split("loss_D = ")[1]) for l in lines])
    flat = lambda m: torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().double()
    return flat(model), flat(model_D), loss_d, pools


def test_image_pool_on_fused_step_matches_autograd_body():
    """ImagePool(pool_size > 0) in run_training (utils/trainer.py:521-556): the
    fused step supplies G's half, D's gradient is recomputed on the pools'
    outputs.  Against the reference's autograd body with the same pool draws
    (Python `random`) and soft labels (torch), the G and D trajectories agree
    to 1e-2 of their movement (Adam steps of ~lr per parameter, fused vs autograd
    rounding), the D loss lines to 1e-4; without the pools D's trajectory is
    visibly different (the pools did swap samples)."""
    g_f, d_f, l_f, pools = _pool_run(3, True)
    g_e, d_e, l_e, _ = _pool_run(3, False)
    g_0, d_0, _, _ = _pool_run(0, True)
    assert pools[0].num_imgs == 3 and pools[1].num_imgs == 3
    G0, D0 = _pool_run(3, True, iters=0)[:2]
    for a, b, a0 in ((g_f, g_e, G0), (d_f, d_e, D0)):
        e = (a - b).norm() / (b - a0).norm()
        assert e < 1e-2, e
    np.testing.assert_allclose(l_f, l_e, rtol=1e-4, atol=1e-6)
    e0 = (d_0 - d_e).norm() / (d_e - D0).norm()
    assert e0 > 0.05, e0


def test_image_pool_on_fused_step_ragged_smaller_batches():
    """the pooled fused step on equal GT / no-GT batches smaller
    than the step it reuses (4, 4, 2, 4, 4, 2 clouds: the 2-cloud pairs run on
    the step built for 4, _pooled_d_grads slicing the step's 2B logits) follows
    the autograd body as the full-batch case does."""
    g_f, d_f, l_f, _ = _pool_run(3, True, sizes=(4, 4, 2))
    g_e, d_e, l_e, _ = _pool_run(3, False, sizes=(4, 4, 2))
    G0, D0 = _pool_run(3, True, iters=0, sizes=(4, 4, 2))[:2]
    for a, b, a0 in ((g_f, g_e, G0), (d_f, d_e, D0)):
        e = (a - b).norm() / (b - a0).norm()
        assert e < 1e-2, e
    np.testing.assert_allclose(l_f, l_e, rtol=1e-4, atol=1e-6)


def _adv_run(tmp_path, use_graph, iters, drop_last, log_every=1):
    import argparse
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import trainer
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    from oracle import pointnet_np as onp
    torch.manual_seed(0)  # the autograd path's dropout / soft labels draw from torch
    lst = _list(tmp_path, ["modelnet_gzip.h5", "modelnet_contig.h5"] * 2)
    gt_rows = np.array([0, 2, 5, 7, 9, 12])
    gt = D.DeviceCloudLoader(D.ModelNetDatasetGT(lst, gt_rows, npoints=32), 4, seed=11,
                             drop_last=drop_last)
    ng = D.DeviceCloudLoader(D.ModelNetDataset_noGT(lst, gt_rows, npoints=32), 4, seed=12,
                             drop_last=drop_last)
    te = D.DeviceCloudLoader(D.ModelNetDatasetGT(lst, None, npoints=32, data_augmentation=False), 4)
    G = onp.make_params(onp.cls_spec(40), seed=31)
    Dp = onp.make_params(onp.disc_spec(40, 1), seed=32, init="xavier")
    model, model_D = pc.PointNetCls(k=40), pc.DeepConvDiscNet(40, 1)
    model.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in G.items()})
    model_D.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in Dp.items()})
    model.cuda()
    model_D.cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999))
    opt_D = torch.optim.Adam(model_D.parameters(), lr=1e-4, betas=(0.9, 0.999))
    args = argparse.Namespace(device="cuda", total_iterations=iters, iter_save_epoch=10 ** 9,
                              iter_test_epoch=10 ** 9, exp_dir=str(tmp_path), tensorboard=False,
                              lambda_cls=1.0, lambda_adv=0.001, batch_size=4, use_graph=use_graph,
                              log_every=log_every)
    log = _Log()
    trainer.run_training(gt, ng, enumerate(gt), enumerate(ng), te, model, model_D,
                         torch.nn.BCEWithLogitsLoss(), torch.nn.CrossEntropyLoss(), opt, opt_D,
                         ImagePool(0), ImagePool(0), log, log, None, args)
    params = torch.cat([p.detach().reshape(-1) for p in list(model.parameters()) +
                        list(model_D.parameters())]).cpu()
    return params, [l for l in log.lines if l.startswith("iter")], opt


@pytest.mark.parametrize("drop_last", [True, False])
def test_graphed_trainer_equals_eager(tmp_path, drop_last):
    """run_training over DeviceCloudLoaders with each iteration's gathers and
    fused step replayed as one HIP graph (the default) equals the eager fused
    loop bitwise: same parameters, same loss lines (read asynchronously) in
    the same order, across epoch wrap-arounds of both loaders (6 GT and 10
    no-GT clouds in batches of 4) and, with drop_last=False, the ragged last
    batches (eager fused step when both are ragged alike, autograd otherwise)."""
    pa, la, opt_a = _adv_run(tmp_path, True, 9, drop_last)
    pb, lb, _ = _adv_run(tmp_path, False, 9, drop_last)
    assert torch.equal(pa, pb)
    assert la == lb and len(la) == 9
    assert all(float(st["step"]) == 9 for st in opt_a.state.values())
    # log_every = 3 logs iterations 0, 3, 6 and trains identically
    pc_, lc, _ = _adv_run(tmp_path, True, 9, drop_last, log_every=3)
    assert torch.equal(pa, pc_) and lc == [la[0], la[3], la[6]]


def _cls_run(tmp_path, use_graph, iters, drop_last):
    import argparse
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import trainer
    from oracle import pointnet_np as onp
    torch.manual_seed(0)
    lst = _list(tmp_path, ["modelnet_gzip.h5", "modelnet_contig.h5"] * 2)
    gt = D.DeviceCloudLoader(D.ModelNetDatasetGT(lst, None, npoints=32), 4, seed=13,
                             drop_last=drop_last)
    te = D.DeviceCloudLoader(D.ModelNetDatasetGT(lst, None, npoints=32, data_augmentation=False), 4)
    G = onp.make_params(onp.cls_spec(40), seed=33)
    model = pc.PointNetCls(k=40)
    model.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in G.items()})
    model.cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999))
    args = argparse.Namespace(device="cuda", total_iterations=iters, iter_save_epoch=10 ** 9,
                              iter_test_epoch=10 ** 9, exp_dir=str(tmp_path), lambda_cls=1.0,
                              use_graph=use_graph, log_every=1, batch_size=4, tensorboard=False)
    log = _Log()
    trainer.run_training_pointnet_cls(gt, enumerate(gt), te, model, torch.nn.CrossEntropyLoss(),
                                      opt, log, log, None, args)
    params = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu()
    return params, [l for l in log.lines if l.startswith("iter")]


@pytest.mark.parametrize("drop_last", [True, False])
def test_graphed_cls_trainer_equals_eager(tmp_path, drop_last):
    """run_training_pointnet_cls over a DeviceCloudLoader on the fused cls step:
    the graphed iteration (the batch gathered by the step's first launch, the
    epilogue in its last) equals the eager loop bitwise - parameters and loss
    lines - across epoch wrap-arounds (10 clouds in batches of 4) and ragged
    batches."""
    pa, la = _cls_run(tmp_path, True, 7, drop_last)
    pb, lb = _cls_run(tmp_path, False, 7, drop_last)
    assert torch.equal(pa, pb)
    assert la == lb and len(la) == 7


def _ft_cls_run(tmp_path, use_graph, iters, drop_last=True):
    import argparse
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import trainer
    from oracle import pointnet_np as onp
    rng = np.random.default_rng(41)
    ds = D.ModelNetDatasetGT.__new__(D.ModelNetDatasetGT)  # in-memory clouds of 256 points
    ds.sample_list, ds.npoints, ds.data_augmentation = None, 256, True
    ds.select_data = rng.uniform(-1, 1, (8, 256, 3)).astype(np.float32)
    ds.select_labels = rng.integers(0, 40, 8).astype(np.int32)
    gt = D.DeviceCloudLoader(ds, 4 if drop_last else 3, seed=11, drop_last=drop_last)
    G = onp.make_params(onp.cls_ft_spec(40), seed=42)
    model = pc.PointNetCls(k=40, feature_transform=True)
    model.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in G.items()})
    model.dropout.p = 0.0  # the graph's and the eager loop's torch.rand draws differ
    model.cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999), capturable=True)
    args = argparse.Namespace(device="cuda", total_iterations=iters, iter_save_epoch=10 ** 9,
                              iter_test_epoch=10 ** 9, exp_dir=str(tmp_path), lambda_cls=1.0,
                              lambda_regu=0.001, use_graph=use_graph, log_every=1, batch_size=4,
                              tensorboard=False)
    log = _Log()
    te = [(torch.from_numpy(ds.select_data[:4].copy()), torch.from_numpy(ds.select_labels[:4].astype(np.int64)))]
    trainer.run_training_pointnet_cls(gt, enumerate(gt), te, model, torch.nn.CrossEntropyLoss(),
                                      opt, log, log, None, args)
    params = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu()
    return params, [l for l in log.lines if l.startswith("iter")], opt


def _ft_adv_run(tmp_path, monkeypatch, use_graph, iters, drop_last):
    """run_training with a feature-transform generator (off the fused step) and
    capturable Adams over in-memory DeviceCloudLoaders (8 GT / 10 no-GT clouds
    of 256 points, batches of 4).  Dropout p = 0 and constant D labels (0.9 /
    0.1 for the soft ones) leave no random draw in the body, so the graphed and
    the eager loop can be compared bitwise."""
    import argparse
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import trainer
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    from oracle import pointnet_np as onp
    monkeypatch.setattr(trainer, "make_D_label", lambda inp, value, device, random=False:
                        torch.full(inp.shape, (0.9 if value else 0.1) if random else float(value),
                                   device=device))
    rng = np.random.default_rng(51)

    def mem(cls, n):
        ds = cls.__new__(cls)
        ds.sample_list, ds.npoints, ds.data_augmentation = None, 256, True
        ds.select_data = rng.uniform(-1, 1, (n, 256, 3)).astype(np.float32)
        if cls is D.ModelNetDatasetGT:
            ds.select_labels = rng.integers(0, 40, n).astype(np.int32)
        return ds
    gds, nds = mem(D.ModelNetDatasetGT, 8), mem(D.ModelNetDataset_noGT, 10)
    gt = D.DeviceCloudLoader(gds, 4, seed=11, drop_last=drop_last)
    ng = D.DeviceCloudLoader(nds, 4, seed=12, drop_last=drop_last)
    G = onp.make_params(onp.cls_ft_spec(40), seed=52)
    Dp = onp.make_params(onp.disc_spec(40, 1), seed=53, init="xavier")
    model, model_D = pc.PointNetCls(k=40, feature_transform=True), pc.DeepConvDiscNet(40, 1)
    model.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in G.items()})
    model_D.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in Dp.items()})
    model.dropout.p = 0.0
    model.cuda()
    model_D.cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999), capturable=True)
    opt_D = torch.optim.Adam(model_D.parameters(), lr=1e-4, betas=(0.9, 0.999), capturable=True)
    args = argparse.Namespace(device="cuda", total_iterations=iters, iter_save_epoch=10 ** 9,
                              iter_test_epoch=10 ** 9, exp_dir=str(tmp_path), tensorboard=False,
                              lambda_cls=1.0, lambda_adv=0.01, batch_size=4, use_graph=use_graph)
    te = [(torch.from_numpy(gds.select_data[:4].copy()),
           torch.from_numpy(gds.select_labels[:4].astype(np.int64)))]
    replays = []
    replay = trainer._GraphedIteration.replay
    monkeypatch.setattr(trainer._GraphedIteration, "replay",
                        lambda self, semi=False: (replays.append(semi), replay(self, semi))[1])
    log = _Log()
    trainer.run_training(gt, ng, enumerate(gt), enumerate(ng), te, model, model_D,
                         torch.nn.BCEWithLogitsLoss(), torch.nn.CrossEntropyLoss(), opt, opt_D,
                         ImagePool(0), ImagePool(0), log, log, None, args)
    params = torch.cat([p.detach().reshape(-1) for p in list(model.parameters()) +
                        list(model_D.parameters())]).cpu()
    grads = torch.cat([p.grad.reshape(-1) for p in list(model.parameters()) +
                       list(model_D.parameters())]).cpu()
    return params, grads, [l for l in log.lines if l.startswith("iter")], (opt, opt_D), len(replays)


@pytest.mark.parametrize("drop_last", [True, False])
def test_graphed_feature_transform_adv_loop_equals_eager(tmp_path, monkeypatch, drop_last):
    """run_training off the fused step (PointNetCls(feature_transform=True)) with
    capturable Adams: each full iteration's gathers + autograd body replayed as
    one HIP graph equals the eager loop bitwise (parameters, the last
    iteration's gradients, loss lines, Adam steps), across epoch wrap-arounds
    and, with drop_last=False, ragged batches run eagerly between replays (the
    graph's gradient buffers rebound after them)."""
    pa, ga, la, opts, na = _ft_adv_run(tmp_path, monkeypatch, True, 7, drop_last)
    pb, gb, lb, _, nb = _ft_adv_run(tmp_path, monkeypatch, False, 7, drop_last)
    # no-GT batches 4, 4 (+ a ragged 2 without drop_last) per epoch
    assert nb == 0 and na == (7 if drop_last else 5)
    assert torch.equal(pa, pb) and torch.equal(ga, gb)
    assert la == lb and len(la) == 7
    for o in opts:
        assert all(float(st["step"]) == 7 for st in o.state.values())


@pytest.mark.parametrize("drop_last", [True, False])
def test_graphed_feature_transform_cls_loop_equals_eager(tmp_path, drop_last):
    """run_training_pointnet_cls with feature_transform=True (not covered by the
    fused cls step) and a capturable Adam over a DeviceCloudLoader: each
    iteration's gather + autograd body replayed as one HIP graph equals the
    eager loop bitwise (parameters, loss / regulariser lines, Adam steps),
    across epoch wrap-arounds (8 clouds, batches of 4; or of 3 with the ragged
    2-cloud batch run eagerly between replays)."""
    pa, la, opt_a = _ft_cls_run(tmp_path, True, 5, drop_last)
    pb, lb, _ = _ft_cls_run(tmp_path, False, 5, drop_last)
    assert torch.equal(pa, pb)
    assert la == lb and len(la) == 5
    assert all(float(st["step"]) == 5 for st in opt_a.state.values())


def _lr_change_run(tmp_path, use_graph, change):
    """run_training over DeviceCloudLoaders for 6 iterations; the test loader
    (iterated by run_testing at i_iter 0, 2, 4) raises both optimizers' lr
    tenfold when it is iterated the second time (a scheduler's effect)."""
    import argparse
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import trainer
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    from oracle import pointnet_np as onp
    lst = _list(tmp_path, ["modelnet_gzip.h5", "modelnet_contig.h5"] * 2)
    gt_rows = np.array([0, 2, 5, 7, 9, 12])
    gt = D.DeviceCloudLoader(D.ModelNetDatasetGT(lst, gt_rows, npoints=32), 4, seed=11, drop_last=True)
    ng = D.DeviceCloudLoader(D.ModelNetDataset_noGT(lst, gt_rows, npoints=32), 4, seed=12,
                             drop_last=True)
    te = D.DeviceCloudLoader(D.ModelNetDatasetGT(lst, None, npoints=32, data_augmentation=False), 4)
    model, model_D = pc.PointNetCls(k=40), pc.DeepConvDiscNet(40, 1)
    model.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in
                           onp.make_params(onp.cls_spec(40), seed=31).items()})
    model_D.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in
                             onp.make_params(onp.disc_spec(40, 1), seed=32, init="xavier").items()})
    model.cuda()
    model_D.cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    opt_D = torch.optim.Adam(model_D.parameters(), lr=1e-4)

    class _Test:
        n = 0

        def __iter__(self):
            _Test.n += 1
            if change and _Test.n == 2:
                for o in (opt, opt_D):
                    o.param_groups[0]["lr"] = 1e-3
            return iter(te)

        def __len__(self):
            return len(te)

    args = argparse.Namespace(device="cuda", total_iterations=6, iter_save_epoch=10 ** 9,
                              iter_test_epoch=2, exp_dir=str(tmp_path), tensorboard=False,
                              lambda_cls=1.0, lambda_adv=0.001, batch_size=4, use_graph=use_graph)
    log = _Log()
    trainer.run_training(gt, ng, enumerate(gt), enumerate(ng), _Test(), model, model_D,
                         torch.nn.BCEWithLogitsLoss(),
                         torch.nn.CrossEntropyLoss(), opt, opt_D, ImagePool(0), ImagePool(0), log,
                         log, None, args)
    return torch.cat([p.detach().reshape(-1) for p in list(model.parameters()) +
                      list(model_D.parameters())]).cpu()


def test_graphed_trainer_follows_an_lr_change(tmp_path):
    """a captured iteration bakes lr / betas / eps in.  When the
    optimizers' lr changes mid-run, the graphed trainer recaptures (and the
    fused step re-reads its hyperparameters), so it stays bitwise the eager
    fused loop, and the change does take effect."""
    a = _lr_change_run(tmp_path, True, True)
    b = _lr_change_run(tmp_path, False, True)
    c = _lr_change_run(tmp_path, True, False)
    assert torch.equal(a, b)
    assert not torch.equal(a, c)
