"""Training / evaluation loops with the reference's signatures
(utils/trainer.py:30-69 run_testing, :72-143 run_testing_seg, :222-308
run_training_pointnet_cls, :310-400 run_training_pointnet_seg, :403-608
run_training, :611-847 run_training_semi).

run_training runs each iteration through the fused native step
(AdvTrainStep: one C-ABI call, no per-op Python) whenever the configuration is
the hot path's (PointNetCls(k=40) + DeepConvDiscNet(40,1), Adam, CE/BCE losses,
ImagePool(0), equal GT/noGT batch sizes); otherwise it runs the reference's
loop body op by op over the same HIP kernels through autograd.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn.functional as F

from .discriminator import DeepConvDiscNet
from .metric import batch_get_iou, object_names
from .pointnet import PointNetCls, feature_transform_regularizer
from .step import AdvTrainStep
from .utils import make_D_label


def run_testing(dataloader, model, criterion, logger, test_iter, writer, args):
    """utils/trainer.py:30-69 (accuracy normalised by batch_size * len(loader),
    as the reference does)."""
    model.eval()
    total_accuracy = 0.0
    total_loss = 0.0
    for batch_idx, data in enumerate(dataloader):
        pts, cls = data
        pts, cls = pts.float().to(args.device), cls.long().to(args.device)
        with torch.set_grad_enabled(False):
            pred, _, _ = model(pts)
            loss = criterion(pred, cls)
        cls = cls.detach().cpu().numpy()
        pred = np.argmax(pred.detach().cpu().numpy(), axis=1)
        total_accuracy += int(np.sum(np.equal(pred, cls)))
        total_loss += loss.item()
    denom = float(args.batch_size * len(dataloader))
    logger.info("Test accuracy: {:.4f} loss: {:.3f}".format(total_accuracy / denom, total_loss / denom))
    if getattr(args, "tensorboard", False) and writer is not None:
        writer.add_scalar("Loss/test_cls", total_loss / denom, test_iter)
        writer.add_scalar("Accuracy/test", total_accuracy / denom, test_iter)
    return total_accuracy / denom, total_loss / denom


# the fused native steps take at most this many clouds per batch (capi.hip:
# pcadv_adv_step / pcadv_cls_step); larger batches run the autograd path
MAX_FUSED_B = 256


def _next(loader, it):
    try:
        _, batch = next(it)
    except StopIteration:
        it = enumerate(loader)
        _, batch = next(it)
    return batch, it


def _fusable(model, model_D, optimizer, optimizer_D, gan_loss, cls_loss, pools, args):
    if not (isinstance(model, PointNetCls) and isinstance(model_D, DeepConvDiscNet)):
        return False
    if model.feature_transform or model.fc3.out_features != 40:
        return False
    if model_D.conv1.in_channels != 40 or model_D.fc.out_features != 1:
        return False
    if str(args.device).split(":")[0] != "cuda":
        return False
    for opt in (optimizer, optimizer_D):
        if type(opt) is not torch.optim.Adam or len(opt.param_groups) != 1:
            return False
        g = opt.param_groups[0]
        if g.get("weight_decay", 0) or g.get("amsgrad") or g.get("maximize"):
            return False
    if type(gan_loss) is not torch.nn.BCEWithLogitsLoss or gan_loss.weight is not None \
            or gan_loss.pos_weight is not None or gan_loss.reduction != "mean":
        return False
    if type(cls_loss) is not torch.nn.CrossEntropyLoss or cls_loss.weight is not None \
            or cls_loss.reduction != "mean" or cls_loss.label_smoothing != 0.0:
        return False
    return all(p.pool_size == 0 for p in pools)


def _save(model, model_D, args, tag):
    torch.save(model.state_dict(), os.path.join(args.exp_dir, "model_{}.pth".format(tag)))
    torch.save(model_D.state_dict(), os.path.join(args.exp_dir, "modelD_{}.pth".format(tag)))


def _semi_fusable(semi_loss):
    return (type(semi_loss) is torch.nn.CrossEntropyLoss and semi_loss.weight is None
            and semi_loss.reduction == "mean" and semi_loss.ignore_index == 255
            and semi_loss.label_smoothing == 0.0)


def _adv_loop(trainloader_gt, trainloader_nogt, trainloader_gt_iter, targetloader_nogt_iter,
              testloader, model, model_D, gan_loss, cls_loss, optimizer, optimizer_D,
              history_pool_gt, history_pool_nogt, train_logger, test_logger, writer, args,
              semi_loss=None):
    """The iteration loop shared by run_training (semi_loss None) and
    run_training_semi (pseudo-label term from iteration semi_start + 1)."""
    gt_label, nogt_label = 1, 0
    max_test_accu = float("-inf")
    max_train_epoch = 0
    fused = _fusable(model, model_D, optimizer, optimizer_D, gan_loss, cls_loss,
                     (history_pool_gt, history_pool_nogt), args)
    if semi_loss is not None:
        fused = fused and _semi_fusable(semi_loss)
    step = None
    log_every = int(getattr(args, "log_every", 1))

    for i_iter in range(args.total_iterations):
        model.train()
        model_D.train()
        batch, trainloader_gt_iter = _next(trainloader_gt, trainloader_gt_iter)
        pts, cls = batch
        pts_nogt, targetloader_nogt_iter = _next(trainloader_nogt, targetloader_nogt_iter)
        pts = pts.float().to(args.device).contiguous()
        cls = cls.long().to(args.device).contiguous()
        pts_nogt = pts_nogt.float().to(args.device).contiguous()
        semi_on = semi_loss is not None and args.semi_start > 0 and i_iter > args.semi_start

        if fused and pts.shape == pts_nogt.shape and pts.shape[0] <= MAX_FUSED_B:
            if step is None or step.N != pts.shape[1] or step.B < pts.shape[0]:
                if step is not None:  # the replacement adopts the Adam state: count included
                    step.sync_optimizer_state()
                step = AdvTrainStep(model, model_D, pts.shape[0], pts.shape[1],
                                    optimizer=optimizer, optimizer_D=optimizer_D,
                                    lambda_cls=args.lambda_cls, lambda_adv=args.lambda_adv,
                                    seed=int(getattr(args, "seed", 0)) + i_iter,
                                    device=args.device,
                                    lambda_semi=float(getattr(args, "lambda_semi", 1.0)),
                                    semi_th=float(getattr(args, "semi_TH", 0.8)))
            losses = step(pts, cls, pts_nogt, semi=semi_on)
            vals = losses.tolist() if (i_iter % log_every == 0) else None
            if vals is not None:
                loss_cls_value, loss_adv_value = vals[0], vals[1]
                loss_D_value = vals[2] + vals[3]
                loss_semi_value = vals[4] if semi_on else 0.0
        else:
            # unequal GT / no-GT batches (a loader's ragged last batch): the
            # reference's body through autograd over the same kernels; the torch
            # optimizers continue from the fused step's Adam state (moments are
            # shared views, the step count is synced in and out)
            if step is not None:
                step.sync_optimizer_state()
            optimizer.zero_grad()
            optimizer_D.zero_grad()
            for param in model_D.parameters():
                param.requires_grad = False
            pred, global_gt, high_feat = model(pts)
            l = cls_loss(pred, cls)
            pred_gt_softmax = F.log_softmax(pred, dim=1)
            pred_nogt, global_nogt, high_feat = model(pts_nogt)
            pred_nogt_softmax = F.log_softmax(pred_nogt, dim=1)
            D_out = model_D(pred_nogt_softmax)
            loss_adv = gan_loss(D_out, make_D_label(D_out, gt_label, args.device, random=False))
            loss = args.lambda_cls * l + args.lambda_adv * loss_adv
            loss_semi_value = 0.0
            if semi_on:  # utils/trainer.py:716-743
                ignore = (D_out <= args.semi_TH).squeeze(1)
                semi_gt = torch.argmax(pred_nogt.detach(), dim=1)
                semi_gt[ignore] = 255
                if int(ignore.sum().item()) < ignore.numel():
                    l_semi = semi_loss(pred_nogt, semi_gt)
                    loss_semi_value = l_semi.item()
                    loss = loss + args.lambda_semi * l_semi
            loss.backward()
            for param in model_D.parameters():
                param.requires_grad = True
            D_out = model_D(history_pool_gt.query(pred_gt_softmax.detach()))
            loss_D1 = gan_loss(D_out, make_D_label(D_out, gt_label, args.device, random=True)) * 0.5
            loss_D1.backward()
            D_out = model_D(history_pool_nogt.query(pred_nogt_softmax.detach()))
            loss_D2 = gan_loss(D_out, make_D_label(D_out, nogt_label, args.device, random=True)) * 0.5
            loss_D2.backward()
            optimizer.step()
            optimizer_D.step()
            if step is not None:
                step.after_torch_step()
            vals = True
            loss_cls_value, loss_adv_value = l.item(), loss_adv.item()
            loss_D_value = loss_D1.item() + loss_D2.item()

        if vals is not None:
            train_logger.info("iter = {0:8d}/{1:8d} loss_cls = {2:.3f} loss_adv = {3:.3f} "
                              "loss_D = {4:.3f}".format(i_iter, args.total_iterations,
                                                        loss_cls_value, loss_adv_value,
                                                        loss_D_value))
            if getattr(args, "tensorboard", False) and writer is not None:
                writer.add_scalar("Loss/train_cls", loss_cls_value, i_iter)
                writer.add_scalar("Loss/train_adv", loss_adv_value, i_iter)
                writer.add_scalar("Loss/train_disc", loss_D_value, i_iter)
                if semi_loss is not None:
                    writer.add_scalar("Loss/train_semi", loss_semi_value, i_iter)

        if i_iter % args.iter_save_epoch == 0:
            if step is not None:
                step.sync_optimizer_state()
            if semi_loss is None:
                tag = i_iter // args.iter_save_epoch
            else:  # trainer.py:789
                tag = int(round(i_iter / len(trainloader_gt)))
            _save(model, model_D, args, "train_epoch_{}".format(tag))
        if i_iter % args.iter_test_epoch == 0:
            curr_accu, _ = run_testing(testloader, model, cls_loss, test_logger, i_iter, writer, args)
            if max_test_accu < curr_accu:
                max_test_accu = curr_accu
                max_train_epoch = i_iter // args.iter_test_epoch
                _save(model, model_D, args, "train_best")

    if step is not None:
        step.sync_optimizer_state()
    if getattr(args, "tensorboard", False) and writer is not None:
        writer.close()
    train_logger.info("Max test accuracy: {:.4f}".format(max_test_accu))
    train_logger.info("Train model is at epoch: {}".format(max_train_epoch))
    return max_test_accu


def run_training(trainloader_gt, trainloader_nogt, trainloader_gt_iter, targetloader_nogt_iter,
                 testloader, model, model_D, gan_loss, cls_loss, optimizer, optimizer_D,
                 history_pool_gt, history_pool_nogt, train_logger, test_logger, writer, args):
    """utils/trainer.py:403-608."""
    return _adv_loop(trainloader_gt, trainloader_nogt, trainloader_gt_iter, targetloader_nogt_iter,
                     testloader, model, model_D, gan_loss, cls_loss, optimizer, optimizer_D,
                     history_pool_gt, history_pool_nogt, train_logger, test_logger, writer, args)


def run_training_semi(trainloader_gt, trainloader_nogt, trainloader_gt_iter,
                      targetloader_nogt_iter, testloader, model, model_D, gan_loss, cls_loss,
                      semi_loss, optimizer, optimizer_D, history_pool_gt, history_pool_nogt,
                      train_logger, test_logger, writer, args):
    """utils/trainer.py:611-847: run_training plus, for i_iter > args.semi_start
    (> 0), lambda_semi x semi_loss(pred_nogt, argmax(pred_nogt)) over the no-GT
    clouds the frozen discriminator scores above args.semi_TH (the rest are
    ignore_index 255; no term when all are ignored).  The fused step computes
    the term on device (k_head_bwd)."""
    return _adv_loop(trainloader_gt, trainloader_nogt, trainloader_gt_iter, targetloader_nogt_iter,
                     testloader, model, model_D, gan_loss, cls_loss, optimizer, optimizer_D,
                     history_pool_gt, history_pool_nogt, train_logger, test_logger, writer, args,
                     semi_loss=semi_loss)


def run_training_pointnet_cls(trainloader_gt, trainloader_gt_iter, testloader, model, cls_loss,
                              optimizer, train_logger, test_logger, writer, args):
    """utils/trainer.py:222-308 (supervised baseline, no discriminator).  With
    PointNetCls(k=40, feature_transform=False), CrossEntropyLoss and Adam on the
    HIP device each iteration is one ClsTrainStep (pcadv_cls_step); otherwise
    (e.g. feature_transform=True, whose regulariser joins the loss) the
    reference's body runs through autograd over the same kernels."""
    from .step import ClsTrainStep
    max_test_accu = float("-inf")
    max_train_epoch = 0
    fused = (isinstance(model, PointNetCls) and not model.feature_transform
             and model.fc3.out_features == 40 and type(optimizer) is torch.optim.Adam
             and len(optimizer.param_groups) == 1
             and not optimizer.param_groups[0].get("weight_decay", 0)
             and not optimizer.param_groups[0].get("amsgrad")
             and type(cls_loss) is torch.nn.CrossEntropyLoss and cls_loss.weight is None
             and cls_loss.reduction == "mean" and cls_loss.label_smoothing == 0.0
             and str(args.device).split(":")[0] == "cuda")
    step = None
    for i_iter in range(args.total_iterations):
        model.train()
        batch, trainloader_gt_iter = _next(trainloader_gt, trainloader_gt_iter)
        pts, cls = batch
        pts, cls = pts.float().to(args.device).contiguous(), cls.long().to(args.device).contiguous()
        l_regu = None
        if fused and pts.shape[0] <= MAX_FUSED_B:
            if step is None or step.N != pts.shape[1] or step.B < pts.shape[0]:
                if step is not None:
                    step.sync_optimizer_state()
                step = ClsTrainStep(model, pts.shape[0], pts.shape[1], optimizer=optimizer,
                                    lambda_cls=args.lambda_cls,
                                    seed=int(getattr(args, "seed", 0)) + i_iter, device=args.device)
            l_value = float(step(pts, cls)[0].item())
        else:
            if step is not None:
                step.sync_optimizer_state()
            optimizer.zero_grad()
            pred, global_gt, high_feat = model(pts)
            l = cls_loss(pred, cls)
            loss = args.lambda_cls * l
            if high_feat is not None:  # feature_transform=True (:256-268)
                l_regu = feature_transform_regularizer(high_feat)
                loss = loss + args.lambda_regu * l_regu
            loss.backward()
            optimizer.step()
            if step is not None:
                step.after_torch_step()
            l_value = l.item()
        train_logger.info("iter = {0:8d}/{1:8d} loss_cls = {2:.3f} loss regu = {3:.3f} ".format(
            i_iter, args.total_iterations, l_value, 0.0 if l_regu is None else l_regu.item()))
        if i_iter % args.iter_save_epoch == 0:
            if step is not None:
                step.sync_optimizer_state()
            torch.save(model.state_dict(), os.path.join(
                args.exp_dir, "model_train_epoch_{}.pth".format(i_iter // len(trainloader_gt))))
        if i_iter % args.iter_test_epoch == 0:
            curr_accu, _ = run_testing(testloader, model, cls_loss, test_logger, i_iter, writer, args)
            if max_test_accu < curr_accu:
                max_test_accu = curr_accu
                max_train_epoch = i_iter // args.iter_test_epoch
                torch.save(model.state_dict(), os.path.join(args.exp_dir, "model_train_best.pth"))
    if step is not None:
        step.sync_optimizer_state()
    train_logger.info("Max test accuracy: {:.4f}".format(max_test_accu))
    train_logger.info("Train model is at epoch: {}".format(max_train_epoch))
    return max_test_accu


def run_testing_seg(dataloader, dataset, model, criterion, logger, test_iter, writer, args):
    """utils/trainer.py:72-143: point accuracy, loss and the category / all-shape
    mean part IoU (the reference's np.object container, removed from numpy,
    becomes a list of lists)."""
    model.eval()
    total_accuracy = 0.0
    total_loss = 0.0
    shape_ious = [[] for _ in object_names]
    for batch_idx, data in enumerate(dataloader):
        pts, cls, seg = data
        pts, cls, seg = pts.float().to(args.device), cls.to(args.device), seg.long().to(args.device)
        with torch.set_grad_enabled(False):
            pred, _ = model(pts, cls)
            loss = criterion(pred, seg)
        pred_seg = pred.max(1)[1]
        total_accuracy += pred_seg.eq(seg).cpu().numpy().sum() / float(args.input_pts)
        total_loss += loss.item()
        p, s_, c = pred_seg.cpu().numpy(), seg.cpu().numpy(), cls[:, 0, :].cpu().numpy()
        for b, iou in enumerate(batch_get_iou(batch_pred=p, batch_seg=s_, batch_cls=c)):
            shape_ious[int(np.argmax(c[b, :]))].append(iou)
    mean_cat = float(np.mean([np.mean(i) for i in shape_ious]))
    mean_all = float(np.mean([i for s in shape_ious for i in s]))
    n = float(len(dataset))
    logger.info("Test accuracy: {:.4f}\tloss: {:.3f}\tcat_iou: {:.4f}\tall_iou: {:.4f}".format(
        total_accuracy / n, total_loss / n, mean_cat, mean_all))
    if getattr(args, "tensorboard", False) and writer is not None:
        writer.add_scalar("Loss/test_cls", total_loss / n, test_iter)
        writer.add_scalar("Accuracy/test", total_accuracy / n, test_iter)
        writer.add_scalar("IoU/test_cat_iou", mean_cat, test_iter)
        writer.add_scalar("IoU/test_all_iou", mean_all, test_iter)
    return total_accuracy / n, total_loss / n, mean_cat, mean_all


def run_training_pointnet_seg(trainloader_gt, trainloader_gt_iter, testloader, testdataset, model,
                              seg_loss, optimizer, train_logger, test_logger, writer, args):
    """utils/trainer.py:310-400.  With PointNetSeg + CrossEntropyLoss + Adam on
    the HIP device each iteration is one SegTrainStep (forward, per-point CE,
    backward into a flat gradient buffer, one Adam launch); otherwise the
    reference's body runs through autograd over the same kernels."""
    from .seg import PointNetSeg, SegTrainStep
    max_test_accu = max_test_cat_iou = max_test_all_iou = float("-inf")
    max_train_epoch = max_train_cat_epoch = max_train_all_epoch = 0
    fused = (isinstance(model, PointNetSeg) and type(optimizer) is torch.optim.Adam
             and len(optimizer.param_groups) == 1
             and not optimizer.param_groups[0].get("weight_decay", 0)
             and not optimizer.param_groups[0].get("amsgrad")
             and type(seg_loss) is torch.nn.CrossEntropyLoss and seg_loss.weight is None
             and seg_loss.reduction == "mean" and seg_loss.ignore_index < 0
             and seg_loss.label_smoothing == 0.0 and str(args.device).split(":")[0] == "cuda")
    step = None
    for i_iter in range(args.total_iterations):
        model.train()
        batch, trainloader_gt_iter = _next(trainloader_gt, trainloader_gt_iter)
        pts, cls, seg = batch
        pts = pts.float().to(args.device).contiguous()
        cls = cls.float().to(args.device).contiguous()
        seg = seg.long().to(args.device).contiguous()
        if fused:
            if step is None:
                step = SegTrainStep(model, optimizer=optimizer, lambda_seg=args.lambda_seg,
                                    device=args.device)
            loss_seg_value = float(step(pts, cls, seg).item())
        else:
            optimizer.zero_grad()
            pred, global_gt = model(pts, cls)
            l = seg_loss(pred, seg)
            loss_seg_value = l.item()
            (args.lambda_seg * l).backward()
            optimizer.step()
        train_logger.info("iter = {0:8d}/{1:8d} loss_seg = {2:.3f} ".format(
            i_iter, args.total_iterations, loss_seg_value))
        if getattr(args, "tensorboard", False) and writer is not None:
            writer.add_scalar("Loss/train_seg", loss_seg_value, i_iter)
        if i_iter % args.iter_save_epoch == 0:
            if step is not None:
                step.sync_optimizer_state()
            torch.save(model.state_dict(), os.path.join(
                args.exp_dir, "model_train_epoch_{}.pth".format(i_iter // len(trainloader_gt))))
        if i_iter % args.iter_test_epoch == 0:
            accu, _, cat_iou, all_iou = run_testing_seg(testloader, testdataset, model, seg_loss,
                                                        test_logger, i_iter, writer, args)
            for tag, val in (("accu", accu), ("cat_iou", cat_iou), ("all_iou", all_iou)):
                best = {"accu": max_test_accu, "cat_iou": max_test_cat_iou,
                        "all_iou": max_test_all_iou}[tag]
                if best < val:
                    ep = i_iter // args.iter_test_epoch
                    if tag == "accu":
                        max_test_accu, max_train_epoch = val, ep
                    elif tag == "cat_iou":
                        max_test_cat_iou, max_train_cat_epoch = val, ep
                    else:
                        max_test_all_iou, max_train_all_epoch = val, ep
                    torch.save(model.state_dict(),
                               os.path.join(args.exp_dir, "model_train_best_{}.pth".format(tag)))
    if step is not None:
        step.sync_optimizer_state()
    if getattr(args, "tensorboard", False) and writer is not None:
        writer.close()
    train_logger.info("=========================")
    train_logger.info("Max test accuracy: {:.4f}, at epoch: {}".format(max_test_accu, max_train_epoch))
    train_logger.info("Max cat mIoU: {:.4f}, at epoch: {}".format(max_test_cat_iou, max_train_cat_epoch))
    train_logger.info("Max all mIoU: {:.4f}, at epoch: {}".format(max_test_all_iou, max_train_all_epoch))
    return max_test_accu, max_test_cat_iou, max_test_all_iou
