"""Capture golden vectors from the reference (run in the build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [/root/reference]

Imports the reference's own modules from /root/reference (read-only; nothing is
copied) and runs them on CPU with deterministic inputs:

* weights come from ``oracle.pointnet_np.make_params`` (numpy PCG64, seeded),
  loaded into the reference models with ``load_state_dict`` - so only seeds are
  stored, never weights;
* stochastic parts are injected: the dropout mask replaces ``model.dropout``
  (models/pointnet.py:194,201) and the soft D labels replace
  ``utils.trainer.make_D_label``'s uniform_ draw (utils/utils.py:28);
* ``run_training`` (utils/trainer.py:403-608) is driven with in-memory loaders.

Outputs small ``.npz`` fixtures next to this script.  The GPU box never sees
the reference; it only sees these fixtures.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import pointnet_np as onp  # noqa: E402

B_SMALL = 4
N_PTS = 1024
SAMPLES = 512
FULL_LIMIT = 16384


def summarize(prefix, arr, out, rng_seed=1234):
    """Full tensor when small; sum / l2 / absmax + fixed-index samples else."""
    a = np.asarray(arr, np.float32)
    if a.size <= FULL_LIMIT:
        out[prefix] = a
        return
    flat = a.reshape(-1)
    idx = np.random.default_rng(rng_seed).choice(flat.size, SAMPLES, replace=False)
    idx.sort()
    out[prefix + ".sum"] = np.float64(flat.astype(np.float64).sum())
    out[prefix + ".l2"] = np.float64(np.sqrt((flat.astype(np.float64) ** 2).sum()))
    out[prefix + ".absmax"] = np.float32(np.abs(flat).max())
    out[prefix + ".idx"] = idx.astype(np.int64)
    out[prefix + ".val"] = flat[idx]


def make_pts(seed, B, N):
    return np.random.default_rng(seed).uniform(-1, 1, (B, N, 3)).astype(np.float32)


def make_mask(rng, B, width=256, p=0.3):
    return (rng.random((B, width)) >= p).astype(np.float32)


def main(ref_root, only=None):
    sys.dont_write_bytecode = True
    sys.path.insert(0, ref_root)
    import torch
    import torch.nn as nn
    from models.pointnet import PointNetCls, PointNetSeg
    from models.discriminator import DeepConvDiscNet
    import utils.trainer as rtrainer
    from utils.image_pool import ImagePool

    torch.set_num_threads(min(8, os.cpu_count() or 1))

    def load(model, params):
        sd = {k: torch.from_numpy(v.copy()) for k, v in params.items()}
        model.load_state_dict(sd)
        return model

    class MaskDropout(nn.Module):
        """Stands in for nn.Dropout(p=0.3) with masks taken from a queue:
        torch computes input * (bernoulli(1-p) / (1-p))."""

        def __init__(self, masks, p=0.3):
            super().__init__()
            self.masks, self.p = masks, p

        def forward(self, x):
            if not self.training:
                return x
            m = torch.from_numpy(self.masks.pop(0))
            return x * (m / (1.0 - self.p))

    # ---------------- G7: feature-transform cls step (run_training_pointnet_cls) ----
    # utils/trainer.py:222-268 with PointNetCls(feature_transform=True): loss =
    # lambda_cls * CE + lambda_regu * feature_transform_regularizer(trans_feat).
    # The reference regularizer moves its identity to CUDA (models/pointnet.py:
    # 345-353); the harness swaps in the same formula with a CPU identity.
    def g7():
        Gf7 = onp.make_params(onp.cls_ft_spec(40), seed=7)
        rng = np.random.default_rng(71)
        pts7 = rng.uniform(-1, 1, (B_SMALL, N_PTS, 3)).astype(np.float32)
        lab7 = rng.integers(0, 40, B_SMALL).astype(np.int64)
        mask7 = make_mask(rng, B_SMALL)
        model = load(PointNetCls(k=40, feature_transform=True), Gf7)
        model.dropout = MaskDropout([mask7.copy()])
        rec = {"cls": [], "reg": []}

        def reg_cpu(trans):
            d = trans.size(1)
            r = torch.mean(torch.norm(torch.bmm(trans, trans.transpose(2, 1)) -
                                      torch.eye(d)[None], dim=(1, 2)))
            rec["reg"].append(float(r.item()))
            return r

        class RecCE(nn.Module):
            def forward(self, a, b):
                r = nn.functional.cross_entropy(a, b)
                rec["cls"].append(float(r.item()))
                return r

        optimizer = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999))
        args = argparse.Namespace(device=torch.device("cpu"), total_iterations=1, lambda_cls=1.0,
                                  lambda_regu=0.001, iter_save_epoch=10 ** 9,
                                  iter_test_epoch=10 ** 9, exp_dir=tempfile.mkdtemp(prefix="g7_"),
                                  tensorboard=False, batch_size=B_SMALL)
        logger = logging.getLogger("golden7")
        logger.addHandler(logging.NullHandler())
        logger.propagate = False
        batch = (torch.from_numpy(pts7), torch.from_numpy(lab7))
        orig = rtrainer.feature_transform_regularizer
        rtrainer.feature_transform_regularizer = reg_cpu
        try:
            rtrainer.run_training_pointnet_cls(
                trainloader_gt=[batch], trainloader_gt_iter=enumerate([batch]),
                testloader=[batch], model=model, cls_loss=RecCE(), optimizer=optimizer,
                train_logger=logger, test_logger=logger, writer=None, args=args)
        finally:
            rtrainer.feature_transform_regularizer = orig
        out = dict(g_seed=7, data_seed=71, B=B_SMALL, N=N_PTS, pts=pts7, labels=lab7,
                   mask=mask7, lambda_cls=1.0, lambda_regu=0.001,
                   loss_cls=np.float64(rec["cls"][0]), reg=np.float64(rec["reg"][0]))
        for name, p in model.named_parameters():
            summarize("grad." + name, p.grad.numpy(), out)
            summarize("param." + name, p.detach().numpy(), out)
        np.savez_compressed(os.path.join(HERE, "g7_cls_ft_step.npz"), **out)

    # ---------------- G8: segmentation training step (run_training_pointnet_seg) ----
    # utils/trainer.py:334-349: pred, _ = model(pts, cls); l = seg_loss(pred, seg)
    # with seg_loss = CrossEntropyLoss() (pointnet/train_pointnet_seg.py:152);
    # (lambda_seg * l).backward(); optimizer.step() with Adam(lr=1e-4).
    def g8():
        Sp = onp.make_params(onp.seg_spec(50), seed=8)
        model = load(PointNetSeg(50), Sp).train()
        B8, N8 = 2, 512
        pts8 = make_pts(81, B8, N8)
        rng8 = np.random.default_rng(82)
        cls8 = np.zeros((B8, 1, 16), np.float32)
        cls8[np.arange(B8), 0, rng8.integers(0, 16, B8)] = 1
        seg8 = rng8.integers(0, 50, (B8, N8)).astype(np.int64)
        opt = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999))
        opt.zero_grad()
        pred, glob = model(torch.from_numpy(pts8), torch.from_numpy(cls8))
        l = torch.nn.CrossEntropyLoss()(pred, torch.from_numpy(seg8))
        (1.0 * l).backward()
        out = dict(s_seed=8, pts_seed=81, cls=cls8, seg=seg8, loss=np.float64(l.item()),
                   gmax=glob.detach().numpy()[:, :, 0])
        summarize("logits", pred.detach().numpy(), out)
        for name, p in model.named_parameters():
            summarize("grad." + name, p.grad.numpy(), out)
        opt.step()
        for name, p in model.named_parameters():
            summarize("param." + name, p.detach().numpy(), out)
        np.savez_compressed(os.path.join(HERE, "g8_seg_step.npz"), **out)

    # ---------------- G9: run_training_semi (pseudo-label step) ----------------
    # utils/trainer.py:611-847 for 3 iterations with semi_start = 1, so the
    # pseudo-label CE (ignore_index=255) joins the generator loss at i_iter 2.
    # semi_TH is set between the middle two D scores of that iteration's no-GT
    # clouds (found with the oracle, which tracks the reference to ~1e-6), so
    # half the clouds are kept and half ignored.
    def g9():
        iters, B, data_seed = 3, 8, 91
        Gp = onp.make_params(onp.cls_spec(40), seed=1)
        Dp = onp.make_params(onp.disc_spec(40, 1), seed=2, init="xavier")
        rng = np.random.default_rng(data_seed)
        batches_gt, batches_ng, masks, soft = [], [], [], []
        for _ in range(iters):
            batches_gt.append((rng.uniform(-1, 1, (B, N_PTS, 3)).astype(np.float32),
                               rng.integers(0, 40, B).astype(np.int64)))
            batches_ng.append(rng.uniform(-1, 1, (B, N_PTS, 3)).astype(np.float32))
            masks.append(make_mask(rng, B))
            masks.append(make_mask(rng, B))
            soft.append(rng.uniform(0.7, 1.05, (B, 1)).astype(np.float32))
            soft.append(rng.uniform(0.0, 0.305, (B, 1)).astype(np.float32))
        # threshold from the oracle's D scores at i_iter 2
        oG = {k: v.copy() for k, v in Gp.items()}
        oD = {k: v.copy() for k, v in Dp.items()}
        aG, aD = onp.Adam(oG), onp.Adam(oD)
        for it in range(2):
            onp.adv_step(oG, oD, aG, aD, batches_gt[it][0], batches_gt[it][1], batches_ng[it],
                         masks[2 * it], masks[2 * it + 1], soft[2 * it], soft[2 * it + 1])
        _, _, _, aux = onp.adv_step(oG, oD, aG, aD, batches_gt[2][0], batches_gt[2][1],
                                    batches_ng[2], masks[4], masks[5], soft[4], soft[5],
                                    apply_adam=False)
        d = np.sort(aux["d_nogt"][:, 0])
        semi_th = float((d[B // 2 - 1] + d[B // 2]) / 2)

        model = load(PointNetCls(k=40, feature_transform=False), Gp)
        model.dropout = MaskDropout([m.copy() for m in masks])
        model_D = load(DeepConvDiscNet(40, 1), Dp)
        soft_q = [x.copy() for x in soft]
        orig = rtrainer.make_D_label

        def make_D_label(input, value, device, random=False):
            if random:
                return torch.from_numpy(soft_q.pop(0)).to(device)
            return orig(input, value, device, random=False)

        rec = {"cls": [], "gan": [], "semi": []}

        class Rec(nn.Module):
            def __init__(self, inner, key):
                super().__init__()
                self.inner, self.key = inner, key

            def forward(self, a, b):
                r = self.inner(a, b)
                rec[self.key].append(float(r.item()))
                return r

        optimizer = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999))
        optimizer_D = torch.optim.Adam(model_D.parameters(), lr=1e-4, betas=(0.9, 0.999))
        tmp = tempfile.mkdtemp(prefix="golden_")
        args = argparse.Namespace(device=torch.device("cpu"), total_iterations=iters,
                                  lambda_cls=1.0, lambda_adv=0.001, lambda_semi=1.0,
                                  semi_start=1, semi_TH=semi_th,
                                  iter_save_epoch=10 ** 9, iter_test_epoch=10 ** 9,
                                  exp_dir=tmp, tensorboard=False, batch_size=B)
        gt_list = [(torch.from_numpy(a), torch.from_numpy(b)) for a, b in batches_gt]
        ng_list = [torch.from_numpy(a) for a in batches_ng]
        logger = logging.getLogger("golden")
        logger.addHandler(logging.NullHandler())
        logger.propagate = False
        rtrainer.make_D_label = make_D_label
        try:
            rtrainer.run_training_semi(
                trainloader_gt=gt_list, trainloader_nogt=ng_list,
                trainloader_gt_iter=enumerate(list(gt_list)),
                targetloader_nogt_iter=enumerate(list(ng_list)),
                testloader=[gt_list[0]], model=model, model_D=model_D,
                gan_loss=Rec(nn.BCEWithLogitsLoss(), "gan"),
                cls_loss=Rec(nn.CrossEntropyLoss(), "cls"),
                semi_loss=Rec(nn.CrossEntropyLoss(ignore_index=255), "semi"),
                optimizer=optimizer, optimizer_D=optimizer_D,
                history_pool_gt=ImagePool(0), history_pool_nogt=ImagePool(0),
                train_logger=logger, test_logger=logger, writer=None, args=args)
        finally:
            rtrainer.make_D_label = orig
        out = dict(iters=iters, data_seed=data_seed, g_seed=1, d_seed=2, B=B, N=N_PTS,
                   semi_start=1, semi_th=np.float64(semi_th), lambda_semi=1.0,
                   semi_ratio=np.float64(0.5))
        cls_train = [rec["cls"][0]] + rec["cls"][2:]
        gan = np.array(rec["gan"]).reshape(iters, 3)
        out["loss_cls"] = np.array(cls_train)
        out["loss_adv"] = gan[:, 0]
        out["loss_D_gt"] = gan[:, 1] * 0.5
        out["loss_D_nogt"] = gan[:, 2] * 0.5
        out["loss_semi"] = np.array(rec["semi"])  # one term: i_iter 2
        for name, p in model.named_parameters():
            summarize("paramG." + name, p.detach().numpy(), out)
        for name, p in model_D.named_parameters():
            summarize("paramD." + name, p.detach().numpy(), out)
        np.savez_compressed(os.path.join(HERE, "g9_semi_step3.npz"), **out)

    # ---------------- G10: host helpers (ImagePool history, init_weights) ----
    # utils/image_pool.py:10-55 with pool_size=3 on seeded Python `random`;
    # utils/model_utils.py:27-58 xavier init of DeepConvDiscNet on a seeded torch RNG
    def g10():
        import random
        from utils.model_utils import init_weights as ref_init_weights
        pool = ImagePool(3)
        random.seed(5)
        xs = np.random.default_rng(101).standard_normal((6, 2, 40)).astype(np.float32)
        outs = [pool.query(torch.from_numpy(x)).detach().numpy() for x in xs]
        out = dict(pool_size=3, random_seed=5, data_seed=101, queries=xs, pool_out=np.stack(outs))
        torch.manual_seed(3)
        md = DeepConvDiscNet(40, 1)
        ref_init_weights(md, "xavier", init_gain=1.0)
        out["torch_seed"] = 3
        for name, p in md.named_parameters():
            summarize("xavier." + name, p.detach().numpy(), out)
        np.savez_compressed(os.path.join(HERE, "g10_host_helpers.npz"), **out)

    # ---------------- G11: configs[1] at full size (B=32, N=1024) ----------
    # run_training_pointnet_cls's iteration (utils/trainer.py:254-268): forward
    # with an injected dropout mask, CrossEntropyLoss, backward
    def g11():
        G11 = onp.make_params(onp.cls_spec(40), seed=3)
        rng = np.random.default_rng(2001)
        B = 32
        pts11 = rng.uniform(-1, 1, (B, N_PTS, 3)).astype(np.float32)
        lab11 = rng.integers(0, 40, B)
        mask11 = make_mask(rng, B)
        model = load(PointNetCls(k=40, feature_transform=False), G11).train()
        model.dropout = MaskDropout([mask11.copy()])
        logits, glob, _ = model(torch.from_numpy(pts11))
        loss = nn.CrossEntropyLoss()(logits, torch.from_numpy(lab11).long())
        loss.backward()
        out = dict(g_seed=3, data_seed=2001, B=B, N=N_PTS, loss=np.float64(loss.item()),
                   logits=logits.detach().numpy(), gmax=glob.detach().numpy()[:, :, 0])
        for name, p in model.named_parameters():
            summarize("grad." + name, p.grad.numpy(), out)
        np.savez_compressed(os.path.join(HERE, "g11_cls_b32.npz"), **out)

    # ---------------- G12: STN3d forward + backward (models/pointnet.py:14-43) ----
    # The 3x3 input transform regressor on the reference layout B x 3 x N, then
    # T.backward(dT) with a seeded dT: the transform, every parameter gradient
    # and the input gradient (returned point-major, B x N x 3).
    def g12():
        from models.pointnet import STN3d
        Sp = onp.make_params(onp.stnkd_spec("", 3), seed=12)
        m = load(STN3d(), Sp)
        rng = np.random.default_rng(121)
        B12 = 4
        pts12 = rng.uniform(-1, 1, (B12, N_PTS, 3)).astype(np.float32)
        dT = rng.normal(0, 1, (B12, 3, 3)).astype(np.float32)
        x = torch.from_numpy(np.ascontiguousarray(pts12.transpose(0, 2, 1))).requires_grad_(True)
        T = m(x)
        T.backward(torch.from_numpy(dT))
        out = dict(s_seed=12, data_seed=121, B=B12, N=N_PTS, trans=T.detach().numpy(),
                   dx=np.ascontiguousarray(x.grad.numpy().transpose(0, 2, 1)))
        for name, p in m.named_parameters():
            summarize("grad." + name, p.grad.numpy(), out)
        np.savez_compressed(os.path.join(HERE, "g12_stn3d.npz"), **out)

    # ---------------- G13: run_training off the fused step ----
    # utils/trainer.py:426-559 for 3 iterations in three configurations:
    #   ft_pool0:    PointNetCls(feature_transform=True) + ImagePool(0)
    #                (the graphed autograd body, trainer._AutogradAdvStep);
    #   plain_pool3: PointNetCls(feature_transform=False) + ImagePool(3) on both
    #                D inputs (the fused step + trainer._pooled_d_grads);
    #   ft_pool3:    both (the eager autograd body, trainer._adv_body).
    # Dropout masks and soft labels injected as in G3; the pools draw from
    # Python `random` seeded with random_seed (utils/image_pool.py:45-47:
    # random.uniform(0, 1), random.randint(0, pool_size - 1)).
    def g13():
        import random
        iters, B, data_seed = 3, B_SMALL, 131
        out = dict(iters=iters, B=B, N=N_PTS, data_seed=data_seed, g_seed=13, d_seed=14,
                   random_seed=1313, lambda_cls=1.0, lambda_adv=0.01)
        rng = np.random.default_rng(data_seed)
        batches_gt, batches_ng, masks, soft = [], [], [], []
        for _ in range(iters):
            batches_gt.append((rng.uniform(-1, 1, (B, N_PTS, 3)).astype(np.float32),
                               rng.integers(0, 40, B).astype(np.int64)))
            batches_ng.append(rng.uniform(-1, 1, (B, N_PTS, 3)).astype(np.float32))
            masks.append(make_mask(rng, B))
            masks.append(make_mask(rng, B))
            soft.append(rng.uniform(0.7, 1.05, (B, 1)).astype(np.float32))
            soft.append(rng.uniform(0.0, 0.305, (B, 1)).astype(np.float32))
        out["pts_gt"] = np.stack([a for a, _ in batches_gt])
        out["labels"] = np.stack([b for _, b in batches_gt])
        out["pts_nogt"] = np.stack(batches_ng)
        out["masks"] = np.stack(masks).reshape(iters, 2, B, 256)
        out["soft"] = np.stack(soft).reshape(iters, 2, B)
        for cfg, ft, pool in (("ft_pool0", True, 0), ("plain_pool3", False, 3),
                              ("ft_pool3", True, 3)):
            Gp = onp.make_params(onp.cls_ft_spec(40) if ft else onp.cls_spec(40), seed=13)
            Dp = onp.make_params(onp.disc_spec(40, 1), seed=14, init="xavier")
            model = load(PointNetCls(k=40, feature_transform=ft), Gp)
            model.dropout = MaskDropout([m.copy() for m in masks])
            model_D = load(DeepConvDiscNet(40, 1), Dp)
            soft_q = [s.copy() for s in soft]
            orig = rtrainer.make_D_label

            def make_D_label(input, value, device, random=False, _q=soft_q):
                if random:
                    return torch.from_numpy(_q.pop(0)).to(device)
                return orig(input, value, device, random=False)

            rec = {"cls": [], "gan": []}

            class Rec(nn.Module):
                def __init__(self, inner, key):
                    super().__init__()
                    self.inner, self.key = inner, key

                def forward(self, a, b):
                    r = self.inner(a, b)
                    rec[self.key].append(float(r.item()))
                    return r

            optimizer = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999))
            optimizer_D = torch.optim.Adam(model_D.parameters(), lr=1e-4, betas=(0.9, 0.999))
            args = argparse.Namespace(device=torch.device("cpu"), total_iterations=iters,
                                      lambda_cls=1.0, lambda_adv=0.01, iter_save_epoch=10 ** 9,
                                      iter_test_epoch=1,
                                      exp_dir=tempfile.mkdtemp(prefix="g13_"), tensorboard=False,
                                      batch_size=B)
            snaps = []

            class SnapTest:
                """run_testing iterates this after every iteration: the
                iteration's gradients (p.grad until the next zero_grad)."""

                def __init__(self, batch):
                    self.batch = batch

                def __iter__(self, _m=model, _d=model_D):
                    snaps.append({("G", n): p.grad.detach().clone() for n, p in _m.named_parameters()}
                                 | {("D", n): p.grad.detach().clone()
                                    for n, p in _d.named_parameters()})
                    return iter([self.batch])

                def __len__(self):
                    return 1
            gt_list = [(torch.from_numpy(a), torch.from_numpy(b)) for a, b in batches_gt]
            ng_list = [torch.from_numpy(a) for a in batches_ng]
            logger = logging.getLogger("golden13")
            logger.addHandler(logging.NullHandler())
            logger.propagate = False
            pools = (ImagePool(pool), ImagePool(pool))
            random.seed(1313)
            rtrainer.make_D_label = make_D_label
            try:
                rtrainer.run_training(
                    trainloader_gt=gt_list, trainloader_nogt=ng_list,
                    trainloader_gt_iter=enumerate(list(gt_list)),
                    targetloader_nogt_iter=enumerate(list(ng_list)),
                    testloader=SnapTest(gt_list[0]), model=model, model_D=model_D,
                    gan_loss=Rec(nn.BCEWithLogitsLoss(), "gan"),
                    cls_loss=Rec(nn.CrossEntropyLoss(), "cls"),
                    optimizer=optimizer, optimizer_D=optimizer_D,
                    history_pool_gt=pools[0], history_pool_nogt=pools[1],
                    train_logger=logger, test_logger=logger, writer=None, args=args)
            finally:
                rtrainer.make_D_label = orig
            assert not masks or len(model.dropout.masks) == 0
            gan = np.array(rec["gan"]).reshape(iters, 3)
            out[cfg + ".feature_transform"] = int(ft)
            out[cfg + ".pool_size"] = pool
            out[cfg + ".loss_cls"] = np.array(rec["cls"][0::2])  # train / test alternate
            out[cfg + ".loss_adv"] = gan[:, 0]
            out[cfg + ".loss_D_gt"] = gan[:, 1] * 0.5
            out[cfg + ".loss_D_nogt"] = gan[:, 2] * 0.5
            if pool:
                out[cfg + ".pool_gt"] = torch.cat(pools[0].images).numpy()
                out[cfg + ".pool_nogt"] = torch.cat(pools[1].images).numpy()
            assert len(snaps) == iters
            for name, p in model.named_parameters():
                summarize(cfg + ".gradG." + name, p.grad.numpy(), out)
                summarize(cfg + ".grad1G." + name, snaps[0][("G", name)].numpy(), out)
                summarize(cfg + ".paramG." + name, p.detach().numpy(), out)
            for name, p in model_D.named_parameters():
                summarize(cfg + ".gradD." + name, p.grad.numpy(), out)
                summarize(cfg + ".grad1D." + name, snaps[0][("D", name)].numpy(), out)
                summarize(cfg + ".paramD." + name, p.detach().numpy(), out)
        np.savez_compressed(os.path.join(HERE, "g13_adv_off_fused.npz"), **out)

    if only == "g13":
        g13()
        return
    if only == "g12":
        g12()
        return
    if only == "g10":
        g10()
        return
    if only == "full":
        g10()
        g11()
    if only == "g9":
        g9()
        return
    if only == "g7":
        g7()
        return
    if only == "g8":
        g8()
        return

    if only != "full":
        # ---------------- G1: cls forward (eval) ----------------
        G = onp.make_params(onp.cls_spec(40), seed=1)
        model = load(PointNetCls(k=40, feature_transform=False), G).eval()
        pts = make_pts(11, B_SMALL, N_PTS)
        am_holder = {}

        def hook(mod, inp, out):
            am_holder["am"] = torch.max(out, 2)[1].detach().numpy().astype(np.int32)

        h = model.feat.conv4.register_forward_hook(hook)
        with torch.no_grad():
            logits, glob, tf = model(torch.from_numpy(pts))
        h.remove()
        np.savez_compressed(os.path.join(HERE, "g1_cls_fwd.npz"), g_seed=1, pts_seed=11,
                            B=B_SMALL, N=N_PTS, logits=logits.numpy(),
                            gmax=glob.numpy()[:, :, 0], argmax=am_holder["am"])

        # ---------------- G2: cls forward+backward (train, injected dropout) ----
        rng = np.random.default_rng(21)
        mask = make_mask(rng, B_SMALL)
        labels = rng.integers(0, 40, B_SMALL)
        model = load(PointNetCls(k=40, feature_transform=False), G).train()
        model.dropout = MaskDropout([mask.copy()])
        logits, glob, _ = model(torch.from_numpy(pts))
        loss = nn.CrossEntropyLoss()(logits, torch.from_numpy(labels).long())
        loss.backward()
        out = dict(g_seed=1, pts_seed=11, mask=mask, labels=labels.astype(np.int64),
                   loss=np.float64(loss.item()), logits=logits.detach().numpy())
        for name, p in model.named_parameters():
            summarize("grad." + name, p.grad.numpy(), out)
        np.savez_compressed(os.path.join(HERE, "g2_cls_bwd.npz"), **out)

    # ---------------- G3: run_training (adversarial step) ----------------
    def run_adv(iters, seed, B=B_SMALL):
        Gp = onp.make_params(onp.cls_spec(40), seed=1)
        Dp = onp.make_params(onp.disc_spec(40, 1), seed=2, init="xavier")
        rng = np.random.default_rng(seed)
        batches_gt, batches_ng, masks, soft = [], [], [], []
        for _ in range(iters):
            batches_gt.append((rng.uniform(-1, 1, (B, N_PTS, 3)).astype(np.float32),
                               rng.integers(0, 40, B).astype(np.int64)))
            batches_ng.append(rng.uniform(-1, 1, (B, N_PTS, 3)).astype(np.float32))
            masks.append(make_mask(rng, B))   # GT pass  (trainer.py:468)
            masks.append(make_mask(rng, B))   # noGT pass (trainer.py:490)
            soft.append(rng.uniform(0.7, 1.05, (B, 1)).astype(np.float32))   # :530-535
            soft.append(rng.uniform(0.0, 0.305, (B, 1)).astype(np.float32))  # :546-551
        model = load(PointNetCls(k=40, feature_transform=False), Gp)
        model.dropout = MaskDropout([m.copy() for m in masks])
        model_D = load(DeepConvDiscNet(40, 1), Dp)
        soft_q = [s.copy() for s in soft]
        orig = rtrainer.make_D_label

        def make_D_label(input, value, device, random=False):
            if random:
                return torch.from_numpy(soft_q.pop(0)).to(device)
            return orig(input, value, device, random=False)

        rec = {"cls": [], "gan": []}

        class Rec(nn.Module):
            def __init__(self, inner, key):
                super().__init__()
                self.inner, self.key = inner, key

            def forward(self, a, b):
                r = self.inner(a, b)
                rec[self.key].append(float(r.item()))
                return r

        optimizer = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999))
        optimizer_D = torch.optim.Adam(model_D.parameters(), lr=1e-4, betas=(0.9, 0.999))
        tmp = tempfile.mkdtemp(prefix="golden_")
        args = argparse.Namespace(device=torch.device("cpu"), total_iterations=iters,
                                  lambda_cls=1.0, lambda_adv=0.001,
                                  iter_save_epoch=10 ** 9, iter_test_epoch=10 ** 9,
                                  exp_dir=tmp, tensorboard=False, batch_size=B)
        tl = [(torch.from_numpy(batches_gt[0][0]), torch.from_numpy(batches_gt[0][1]))]
        logger = logging.getLogger("golden")
        logger.addHandler(logging.NullHandler())
        logger.propagate = False
        rtrainer.make_D_label = make_D_label
        try:
            rtrainer.run_training(
                trainloader_gt=[(torch.from_numpy(a), torch.from_numpy(b)) for a, b in batches_gt],
                trainloader_nogt=[torch.from_numpy(a) for a in batches_ng],
                trainloader_gt_iter=enumerate([(torch.from_numpy(a), torch.from_numpy(b))
                                               for a, b in batches_gt]),
                targetloader_nogt_iter=enumerate([torch.from_numpy(a) for a in batches_ng]),
                testloader=tl, model=model, model_D=model_D,
                gan_loss=Rec(nn.BCEWithLogitsLoss(), "gan"),
                cls_loss=Rec(nn.CrossEntropyLoss(), "cls"),
                optimizer=optimizer, optimizer_D=optimizer_D,
                history_pool_gt=ImagePool(0), history_pool_nogt=ImagePool(0),
                train_logger=logger, test_logger=logger, writer=None, args=args)
        finally:
            rtrainer.make_D_label = orig
        return dict(batches_gt=batches_gt, batches_ng=batches_ng, masks=masks, soft=soft,
                    rec=rec, model=model, model_D=model_D)

    # (iters, file, B): the B=32 one is BASELINE configs[2]'s full per-GPU batch
    g3_cases = ((1, "g3_adv_step1.npz", B_SMALL), (3, "g3_adv_step3.npz", B_SMALL),
                (1, "g3_adv_step1_b32.npz", 32))
    if only == "full":
        g3_cases = g3_cases[2:]
    for iters, fname, Bc in g3_cases:
        r = run_adv(iters, seed=31, B=Bc)
        out = dict(iters=iters, data_seed=31, g_seed=1, d_seed=2, B=Bc, N=N_PTS)
        # cls criterion: index 0 is the train step, index 1 the iter-0 test pass
        cls_train = [r["rec"]["cls"][0]] + r["rec"]["cls"][2:]
        gan = np.array(r["rec"]["gan"]).reshape(iters, 3)
        out["loss_cls"] = np.array(cls_train)
        out["loss_adv"] = gan[:, 0]
        out["loss_D_gt"] = gan[:, 1] * 0.5
        out["loss_D_nogt"] = gan[:, 2] * 0.5
        if iters == 1:
            for name, p in r["model"].named_parameters():
                summarize("gradG." + name, p.grad.numpy(), out)
            for name, p in r["model_D"].named_parameters():
                summarize("gradD." + name, p.grad.numpy(), out)
        for name, p in r["model"].named_parameters():
            summarize("paramG." + name, p.detach().numpy(), out)
        for name, p in r["model_D"].named_parameters():
            summarize("paramD." + name, p.detach().numpy(), out)
        np.savez_compressed(os.path.join(HERE, fname), **out)
    if only == "full":
        return

    # ---------------- G4: discriminator fwd/bwd ----------------
    Dp = onp.make_params(onp.disc_spec(40, 1), seed=2, init="xavier")
    rng = np.random.default_rng(41)
    x = onp.log_softmax(rng.normal(0, 3, (32, 40)).astype(np.float32))
    dout = rng.normal(0, 1, (32, 1)).astype(np.float32)
    md = load(DeepConvDiscNet(40, 1), Dp)
    xt = torch.from_numpy(x).requires_grad_(True)
    o = md(xt)
    o.backward(torch.from_numpy(dout))
    out = dict(d_seed=2, x=x, dout=dout, out=o.detach().numpy(), dx=xt.grad.numpy())
    for name, p in md.named_parameters():
        summarize("grad." + name, p.grad.numpy(), out)
    np.savez_compressed(os.path.join(HERE, "g4_disc.npz"), **out)

    # ---------------- G5: T-Net feature transform (eval) ----------------
    Gf = onp.make_params(onp.cls_ft_spec(40), seed=5)
    mf = load(PointNetCls(k=40, feature_transform=True), Gf).eval()
    pts5 = make_pts(51, 2, N_PTS)
    with torch.no_grad():
        lg, gl, trans = mf(torch.from_numpy(pts5))
        d = trans.size(1)
        reg = torch.mean(torch.norm(torch.bmm(trans, trans.transpose(2, 1)) -
                                    torch.eye(d)[None], dim=(1, 2)))
    np.savez_compressed(os.path.join(HERE, "g5_tnet.npz"), g_seed=5, pts_seed=51,
                        logits=lg.numpy(), gmax=gl.numpy()[:, :, 0], trans=trans.numpy(),
                        reg=np.float64(reg.item()))

    g7()

    # ---------------- G6: segmentation forward ----------------
    Sp = onp.make_params(onp.seg_spec(50), seed=6)
    ms = load(PointNetSeg(50), Sp).eval()
    pts6 = make_pts(61, 2, 2048)
    cls = np.zeros((2, 1, 16), np.float32)
    cls[0, 0, 3] = 1
    cls[1, 0, 11] = 1
    with torch.no_grad():
        so, sg = ms(torch.from_numpy(pts6), torch.from_numpy(cls))
    out = dict(s_seed=6, pts_seed=61, cls=cls, gmax=sg.numpy()[:, :, 0])
    summarize("out", so.numpy(), out)
    np.savez_compressed(os.path.join(HERE, "g6_seg_fwd.npz"), **out)
    g8()
    g9()
    g10()
    g11()
    g12()

    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("ref_root", nargs="?", default="/root/reference")
    ap.add_argument("--only", default=None, help="g7, g8, g9, g10, g12 or g13: regenerate only that "
                    "fixture; full: g10, g11 and the B=32 g3")
    a = ap.parse_args()
    main(a.ref_root, a.only)
