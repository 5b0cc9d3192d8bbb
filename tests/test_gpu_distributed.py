"""The split adversarial step behind the overlapped data-parallel all-reduce
(pcadv_adv_args.part): part 1 (everything before the feature backward) then
part 2 (the feature backward) must equal the whole step bitwise, and the
bucketed all-reduce must give the same replicas as the single all-reduce.

The multi-rank case runs two gloo ranks on the one GPU of the box (RCCL needs
one device per rank); the gloo all-reduce of device tensors is the same
arithmetic on the same buckets as RCCL's.
"""
import os
import re
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, N = 8, 256


def _models(dev):
    import adversarial_learning_on_pointclouds_amd as pc
    torch.manual_seed(0)
    return pc.PointNetCls(k=40).to(dev), pc.DeepConvDiscNet(40, 1).to(dev)


def _batch(dev, seed, b=B):
    g = torch.Generator().manual_seed(seed)
    pg = (torch.rand(b, N, 3, generator=g) * 2 - 1).to(dev)
    pn = (torch.rand(b, N, 3, generator=g) * 2 - 1).to(dev)
    lab = torch.randint(0, 40, (b,), generator=g).to(dev)
    return pg, lab, pn


def test_parts_equal_whole_step():
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
    dev = torch.device("cuda:0")
    outs = []
    for split in (False, True):
        m, d = _models(dev)
        st = AdvTrainStep(m, d, B, N, seed=7, device=dev)
        for k in range(3):
            pg, lab, pn = _batch(dev, 10 + k)
            if split:
                st(pg, lab, pn, apply_adam=False, part=1)
                st(pg, lab, pn, apply_adam=True, part=2)
            else:
                st(pg, lab, pn)
        torch.cuda.synchronize()
        outs.append((st.grad_flat.clone(), st.g_param.clone(), st.d_param.clone(),
                     st.losses.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_split_adam_equals_whole_adam():
    """adam(part=1) then adam(part=2) (the early bucket's parameters updated
    beside the late all-reduce) equals adam() bitwise, over three steps."""
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
    dev = torch.device("cuda:0")
    outs = []
    for split in (False, True):
        m, d = _models(dev)
        st = AdvTrainStep(m, d, B, N, seed=7, device=dev)
        for k in range(3):
            st.grads(*_batch(dev, 20 + k))
            if split:
                st.adam(part=1)
                st.adam(part=2)
            else:
                st.adam()
        torch.cuda.synchronize()
        outs.append((st.g_param.clone(), st.g_m.clone(), st.g_v.clone(), st.d_param.clone(),
                     st.d_m.clone(), st.d_v.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    with pytest.raises(RuntimeError):
        st.adam(part=3)


def test_part_graphs_equal_whole_graph():
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
    dev = torch.device("cuda:0")
    pg, lab, pn = _batch(dev, 3)
    res = []
    for split in (False, True):
        m, d = _models(dev)
        st = AdvTrainStep(m, d, B, N, seed=7, device=dev)
        if split:
            g1 = st.capture_on(pg, lab, pn, apply_adam=False, part=1)
            g2 = st.capture_on(pg, lab, pn, apply_adam=True, part=2)
            for _ in range(2):
                g1.replay()
                g2.replay()
        else:
            g = st.capture_on(pg, lab, pn)
            for _ in range(2):
                g.replay()
        torch.cuda.synchronize()
        res.append((st.g_param.clone(), st.d_param.clone(), st.losses.clone()))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from adversarial_learning_on_pointclouds_amd.distributed import DataParallelAdvStep
        from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        for overlap in (False, True):
            m, d = _models(dev)
            st = AdvTrainStep(m, d, B, N, seed=7 + rank, device=dev)
            dp = DataParallelAdvStep(st, overlap=overlap)
            graph = dp.capture(*_batch(dev, 40 + rank))
            for k in range(2):
                dp(*_batch(dev, 20 + 2 * k + rank))   # eager
                graph.replay()                        # captured halves around the all-reduce
            torch.cuda.synchronize()
            np.save(os.path.join(out_dir, f"g{rank}_{int(overlap)}.npy"), st.g_param.cpu().numpy())
            np.save(os.path.join(out_dir, f"d{rank}_{int(overlap)}.npy"), st.d_param.cpu().numpy())
    finally:
        dist.destroy_process_group()


def test_bucketed_allreduce_matches_single(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=2, join=True)
    for name in ("g", "d"):
        ref = np.load(tmp_path / f"{name}0_0.npy")
        for rank in (0, 1):
            for ov in (0, 1):
                got = np.load(tmp_path / f"{name}{rank}_{ov}.npy")
                assert np.array_equal(got, ref), (name, rank, ov)


# ---------------------------------------------------------------------------
# configs[4]: the data-parallel step on the HIP path vs the single-process
# oracle on the global batch (models/pointnet.py:109-137, utils/trainer.py:426-559)
# ---------------------------------------------------------------------------

DP_B, DP_N = 32, 2048  # configs[4]'s per-rank shape (B=256 global over 8 ranks)


def _global_batch(world):
    rng = np.random.default_rng(4242)
    Bg = DP_B * world
    pg = rng.uniform(-1, 1, (Bg, DP_N, 3)).astype(np.float32)
    lab = rng.integers(0, 40, Bg)
    pn = rng.uniform(-1, 1, (Bg, DP_N, 3)).astype(np.float32)
    m1 = (rng.random((Bg, 256)) >= 0.3).astype(np.float32)
    m2 = (rng.random((Bg, 256)) >= 0.3).astype(np.float32)
    y1 = rng.uniform(0.7, 1.05, (Bg, 1)).astype(np.float32)
    y2 = rng.uniform(0.0, 0.305, (Bg, 1)).astype(np.float32)
    return pg, lab, pn, m1, m2, y1, y2


def _dp_oracle_worker(rank, port, out_dir, world):
    """One rank: the real AdvTrainStep (HIP) on its slice of the global batch,
    the bucketed all-reduce (overlap on), the replicated Adam."""
    import torch.distributed as dist
    from oracle import pointnet_np as onp
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import adversarial_learning_on_pointclouds_amd as pc
        from adversarial_learning_on_pointclouds_amd.distributed import DataParallelAdvStep
        from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        m = pc.PointNetCls(k=40)
        m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in
                           onp.make_params(onp.cls_spec(40), seed=5).items()})
        d = pc.DeepConvDiscNet(40, 1)
        d.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in
                           onp.make_params(onp.disc_spec(40, 1), seed=6, init="xavier").items()})
        m.to(dev)
        d.to(dev)
        st = AdvTrainStep(m, d, DP_B, DP_N, device=dev)
        dp = DataParallelAdvStep(st, overlap=True)
        sl = slice(rank * DP_B, (rank + 1) * DP_B)
        t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a[sl])).to(dev, dt)
        pg, lab, pn, m1, m2, y1, y2 = _global_batch(world)
        losses = dp(t(pg), t(lab, torch.int64), t(pn), masks=(t(m1), t(m2)), soft=(t(y1), t(y2)))
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), losses=losses.cpu().numpy(),
                 grad=st.grad_flat.cpu().numpy(), g=st.g_param.cpu().numpy(),
                 d=st.d_param.cpu().numpy(),
                 **{"grad." + k: p.grad.cpu().numpy() for k, p in m.named_parameters()},
                 **{"gradD." + k: p.grad.cpu().numpy() for k, p in d.named_parameters()},
                 **{"param." + k: p.detach().cpu().numpy() for k, p in m.named_parameters()},
                 **{"paramD." + k: p.detach().cpu().numpy() for k, p in d.named_parameters()})
    finally:
        dist.destroy_process_group()


def test_dp_two_ranks_hip_step_vs_global_oracle(tmp_path):
    """Two ranks (gloo, sharing the box's GPU), each the real HIP step at
    configs[4]'s per-rank shape, all-reduced: both replicas bitwise equal, and
    the averaged gradients / updated parameters equal the single-process oracle
    step on the 2B global batch (per-tensor relative gradient tolerance)."""
    import torch.multiprocessing as mp
    from oracle import pointnet_np as onp
    from golden_util import assert_grad_close, rel_err
    world = 2
    mp.spawn(_dp_oracle_worker, args=(_free_port(), str(tmp_path), world), nprocs=world, join=True)
    r0, r1 = (dict(np.load(tmp_path / f"r{r}.npz")) for r in range(world))
    for k in ("grad", "g", "d"):
        assert np.array_equal(r0[k], r1[k]), k
    G = onp.make_params(onp.cls_spec(40), seed=5)
    D = onp.make_params(onp.disc_spec(40, 1), seed=6, init="xavier")
    pg, lab, pn, m1, m2, y1, y2 = _global_batch(world)
    ref, gG, gD, _ = onp.adv_step(G, D, onp.Adam(G), onp.Adam(D), pg, lab, pn, m1, m2, y1, y2)
    want = [ref["loss_cls"], ref["loss_adv"], ref["loss_D_gt"], ref["loss_D_nogt"]]
    got = (r0["losses"][:4] + r1["losses"][:4]) / 2  # each rank reports its own shard's means
    assert np.allclose(got, want, atol=1e-4), (got, want)
    for k in gG:
        assert_grad_close(r0["grad." + k], gG[k], k)
        assert rel_err(r0["param." + k], G[k]) < 1e-5, k
    for k in gD:
        assert_grad_close(r0["gradD." + k], gD[k], k)
        assert rel_err(r0["paramD." + k], D[k]) < 1e-5, k


def _rccl_worker(rank, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from adversarial_learning_on_pointclouds_amd.distributed import DataParallelAdvStep
        from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
        res = {}
        for mode in ("plain", "eager", "graphs", "single", "b_eager", "b_graphs", "b_single"):
            m, d = _models(dev)
            st = AdvTrainStep(m, d, B, N, seed=7, device=dev)
            if mode == "plain":
                for k in range(3):
                    st(*_batch(dev, 60 + k))
            else:
                dp = DataParallelAdvStep(st, overlap=mode.startswith("b_"))
                assert dp._split() == mode.startswith("b_")
                if mode.endswith("eager"):
                    for k in range(3):
                        dp(*_batch(dev, 60 + k))
                else:
                    bufs = _batch(dev, 60)
                    graph = dp.capture(*bufs) if mode.endswith("graphs") else dp.capture_single(*bufs)
                    for k in range(3):
                        for dst, src in zip(bufs, _batch(dev, 60 + k)):
                            dst.copy_(src)
                        graph.replay()
            torch.cuda.synchronize()
            res[mode] = np.concatenate([st.g_param.cpu().numpy(), st.d_param.cpu().numpy(),
                                        st.losses.cpu().numpy()])
        np.savez(os.path.join(out_dir, "rccl.npz"), **res)
    finally:
        dist.destroy_process_group()


def test_rccl_data_parallel_paths_single_rank(tmp_path):
    """Every RCCL code path of DataParallelAdvStep on a one-rank RCCL group,
    where the average is the identity, so three steps must equal the plain
    step bitwise: the default single all-reduce (eager; as graphs around the
    collective; as ONE graph with the collective captured, the bench's and the
    trainer's form) and the round-5 bucketed, overlapped all-reduce
    (b_*: ReduceOp.AVG with async_op on RCCL's stream, the two buckets around
    the feature backward).  Checks the stream ordering of every form (a missed
    wait shows as a race on the gradient buffer)."""
    import torch.multiprocessing as mp
    mp.spawn(_rccl_worker, args=(_free_port(), str(tmp_path)), nprocs=1, join=True)
    r = dict(np.load(tmp_path / "rccl.npz"))
    for mode in ("eager", "graphs", "single", "b_eager", "b_graphs", "b_single"):
        assert np.array_equal(r["plain"], r[mode]), mode


# ---------------------------------------------------------------------------
# Data parallelism as a library feature: run_training over
# rank-sharded DeviceCloudLoaders equals the one-process trainer on the global
# batch, device RNG on (jitter, dropout masks, soft D labels keyed by global rows)
# ---------------------------------------------------------------------------

H5 = os.path.join(os.path.dirname(__file__), "golden", "h5")


def _trainer_run(out, rank, world, B, iters, tmp, semi=False):
    import argparse
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import dataset as D
    from adversarial_learning_on_pointclouds_amd import trainer
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    from oracle import pointnet_np as onp
    lst = os.path.join(tmp, f"files{rank}.txt")
    with open(lst, "w") as f:
        f.write("".join(os.path.join(H5, n) + "\n" for n in ["modelnet_gzip.h5", "modelnet_contig.h5"] * 4))
    gt_rows = np.arange(0, 32, 2)
    kw = dict(rank=rank, world_size=world) if world > 1 else {}
    gt = D.DeviceCloudLoader(D.ModelNetDatasetGT(lst, gt_rows, npoints=32), B, seed=11,
                             drop_last=True, **kw)
    ng = D.DeviceCloudLoader(D.ModelNetDataset_noGT(lst, gt_rows, npoints=32), B, seed=12,
                             drop_last=True, **kw)
    te = D.DeviceCloudLoader(D.ModelNetDatasetGT(lst, None, npoints=32, data_augmentation=False), 4,
                             rank=0, world_size=1)
    model, model_D = pc.PointNetCls(k=40), pc.DeepConvDiscNet(40, 1)
    model.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in
                           onp.make_params(onp.cls_spec(40), seed=31).items()})
    model_D.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in
                             onp.make_params(onp.disc_spec(40, 1), seed=32, init="xavier").items()})
    model.cuda()
    model_D.cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, betas=(0.9, 0.999))
    opt_D = torch.optim.Adam(model_D.parameters(), lr=1e-3, betas=(0.9, 0.999))
    args = argparse.Namespace(device="cuda", total_iterations=iters, iter_save_epoch=10 ** 9,
                              iter_test_epoch=10 ** 9, exp_dir=tmp, tensorboard=False,
                              lambda_cls=1.0, lambda_adv=0.01, batch_size=B, seed=3)

    class _Log:
        def __init__(self):
            self.lines = []

        def info(self, s):
            self.lines.append(s)

    log = _Log()
    if semi:
        args.semi_start, args.semi_TH, args.lambda_semi = 1, 0.5, 1.0
        trainer.run_training_semi(gt, ng, enumerate(gt), enumerate(ng), te, model, model_D,
                                  torch.nn.BCEWithLogitsLoss(), torch.nn.CrossEntropyLoss(),
                                  torch.nn.CrossEntropyLoss(ignore_index=255), opt, opt_D,
                                  ImagePool(0), ImagePool(0), log, log, None, args)
    else:
        trainer.run_training(gt, ng, enumerate(gt), enumerate(ng), te, model, model_D,
                             torch.nn.BCEWithLogitsLoss(),
                             torch.nn.CrossEntropyLoss(), opt, opt_D, ImagePool(0), ImagePool(0),
                             log, log, None, args)
    params = torch.cat([p.detach().reshape(-1) for p in list(model.parameters()) +
                        list(model_D.parameters())]).cpu().numpy()
    loss = np.array([[float(x) for x in re.findall(r"= +([-0-9.]+)", l)[1:]]
                     for l in log.lines if l.startswith("iter")])
    np.savez(out, params=params, loss=loss)


def _dp_trainer_worker(rank, port, tmp, world, B, iters, semi=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        if semi:
            try:
                _trainer_run(os.path.join(tmp, f"dp{rank}.npz"), rank, world, B, iters, tmp,
                             semi=True)
            except NotImplementedError as e:
                with open(os.path.join(tmp, f"semi_refused{rank}.txt"), "w") as f:
                    f.write(str(e))
        else:
            _trainer_run(os.path.join(tmp, f"dp{rank}.npz"), rank, world, B, iters, tmp)
    finally:
        dist.destroy_process_group()


def test_dp_trainer_equals_global_batch_trainer(tmp_path):
    """Two ranks (gloo over the box's one GPU; unmeasured on a multi-GPU node)
    run run_training over DeviceCloudLoader(..., world_size=2) shards of 4 + 4
    clouds with device RNG on (jitter, dropout p = 0.3, soft D labels): the
    replicas stay bitwise identical and equal the one-process trainer on the
    8 + 8-cloud global batch (same loader and step seeds) to f32 rounding over
    5 iterations across an epoch wrap; the logged losses are the global
    batch's.  Without the global-row RNG keying the ranks would draw the same
    masks and labels for their local rows and the trajectories would part."""
    import torch.multiprocessing as mp
    world, B, iters = 2, 4, 5
    mp.spawn(_dp_trainer_worker, args=(_free_port(), str(tmp_path), world, B, iters), nprocs=world,
             join=True)
    r0, r1 = (dict(np.load(tmp_path / f"dp{r}.npz")) for r in range(world))
    assert np.array_equal(r0["params"], r1["params"])
    _trainer_run(str(tmp_path / "one.npz"), 0, 1, world * B, iters, str(tmp_path))
    one = dict(np.load(tmp_path / "one.npz"))
    p0 = _initial_params()
    moved = np.abs(one["params"] - p0).max()
    assert moved > 1e-3  # five Adam steps at lr 1e-3
    assert np.abs(r0["params"] - one["params"]).max() < 1e-3 * moved, \
        np.abs(r0["params"] - one["params"]).max()
    assert r0["loss"].shape == one["loss"].shape == (iters, 3)
    np.testing.assert_allclose(r0["loss"], one["loss"], rtol=2e-3, atol=2e-3)


def test_dp_semi_refused(tmp_path):
    """run_training_semi over sharded loaders is refused loudly:
    k_head_bwd normalises the pseudo-label CE by each rank's own kept count, so
    the averaged gradient would not be the global batch's."""
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_dp_trainer_worker, args=(_free_port(), str(tmp_path), world, 4, 3, True),
             nprocs=world, join=True)
    for r in range(world):
        assert "pseudo-label" in (tmp_path / f"semi_refused{r}.txt").read_text()


def _initial_params():
    from oracle import pointnet_np as onp
    return np.concatenate([v.reshape(-1) for v in list(onp.make_params(onp.cls_spec(40), seed=31).values())
                           + list(onp.make_params(onp.disc_spec(40, 1), seed=32,
                                                  init="xavier").values())]).astype(np.float32)
