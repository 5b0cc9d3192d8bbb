"""Data-parallel adversarial step: one process per GPU, RCCL over xGMI.

The reference is single-process (train_classification.py:93); the north star
adds data parallelism.  Clouds are independent, so each rank runs the fused
step on its own B-cloud shards of the GT and noGT batches; the only exchange
is ONE all-reduce(AVG) of the concatenated generator + discriminator gradient
buffer (811 240 + 238 785 fp32 = 4.2 MB) between backward and the replicated
Adam updates.  With equal shards this equals the single-process step on the
global batch, since CE/BCE are batch means (mean of per-rank means).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def _avg_(t, group=None):
    if dist.get_backend(group) == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group)
    else:  # gloo has no AVG
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.div_(dist.get_world_size(group))


class DataParallelAdvStep:
    """Wraps an AdvTrainStep-like object exposing grads(), adam(), grad_flat,
    g_param, d_param and losses."""

    def __init__(self, step, group=None, broadcast_params=True):
        self.step, self.group = step, group
        if broadcast_params:  # identical initial weights on every rank
            dist.broadcast(step.g_param, src=0, group=group)
            dist.broadcast(step.d_param, src=0, group=group)

    def __call__(self, pts_gt, labels, pts_nogt, masks=None, soft=None, semi=False):
        # semi: each rank's pseudo-label CE is the mean over its own kept clouds,
        # so the averaged gradient weights ranks equally (the global-batch mean
        # would weight them by their kept counts)
        self.step.grads(pts_gt, labels, pts_nogt, masks, soft, semi=semi)
        _avg_(self.step.grad_flat, self.group)
        self.step.adam()
        return self.step.losses

    def capture(self, pts_gt, labels, pts_nogt):
        """HIP graphs for the compute halves around the (eager) all-reduce."""
        s = self.step
        g_fwd = s.capture_on(pts_gt, labels, pts_nogt, apply_adam=False)
        saved = s._snapshot()
        g_adam = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(device=s.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            s.adam()
        torch.cuda.current_stream().wait_stream(side)
        with torch.cuda.graph(g_adam):
            s.adam()
        torch.cuda.synchronize()
        s._restore(saved)
        return _DPGraph(g_fwd, g_adam, s, self.group)


class _DPGraph:
    def __init__(self, g_fwd, g_adam, step, group):
        self.g_fwd, self.g_adam, self.step, self.group = g_fwd, g_adam, step, group

    def replay(self):
        self.g_fwd.replay()
        _avg_(self.step.grad_flat, self.group)
        self.g_adam.replay()
        return self.step.losses
