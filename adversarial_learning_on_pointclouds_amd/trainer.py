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

import collections
import contextlib
import os

import numpy as np
import torch
import torch.nn.functional as F

from .discriminator import DeepConvDiscNet
from .metric import batch_get_iou, object_names
from .pointnet import PointNetCls, feature_transform_regularizer
from ._lib import D_LAYOUT
from .dataset import gather_at_multi
from .step import AdvFtTrainStep, AdvTrainStep, _views
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


class _LossRing:
    """The per-iteration loss lines of the training loops (utils/trainer.py:
    561-572) without a host sync per iteration.  Each fused iteration's device
    loss vector goes into slot (count % slots) of a device ring
    (pcadv_iter_epilogue: inside the iteration's graph when it is replayed);
    every slots / 2 iterations one asynchronous copy of the ring to pinned
    host memory is queued, and the lines are emitted in iteration order once
    a copy has landed (polled every iteration; drained before test passes,
    checkpoints, autograd iterations and at the end).  The lines and scalars
    are the reference's, written a few iterations late."""

    def __init__(self, emit, nl, device, slots=64):
        from . import _lib
        self.lib = _lib.load()
        self.emit, self.nl, self.slots, self.half = emit, nl, slots, slots // 2
        self.ring = torch.zeros(slots, nl, device=device)
        self.count = torch.zeros(1, dtype=torch.int32, device=device)
        self.n_written = 0          # host mirror of *count
        self.pending = []           # (slot, i_iter, extra) written, not yet copied
        self.inflight = collections.deque()
        self.free = []

    def write(self, losses, counters=None, ncounters=0):
        """Enqueue the epilogue: losses -> ring slot, counters[0:ncounters] += 1."""
        from ._lib import check, stream_ptr
        import ctypes
        P = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
        check(self.lib.pcadv_iter_epilogue(P(counters), ncounters, P(losses), self.nl,
                                           P(self.ring), self.slots, P(self.count), stream_ptr()),
              "pcadv_iter_epilogue")

    def record(self, i_iter, extra, log=True):
        """After each fused iteration (its epilogue wrote the next slot)."""
        slot = self.n_written % self.slots
        self.n_written += 1
        if log:
            self.pending.append((slot, i_iter, extra))
        if self.n_written % self.half == 0:
            self.flush()
        self.poll()

    def flush(self):
        if not self.pending:
            return
        if self.free:
            buf, ev = self.free.pop()
        else:
            buf, ev = torch.empty(self.slots, self.nl, pin_memory=True), torch.cuda.Event()
        buf.copy_(self.ring, non_blocking=True)  # stream-ordered before any later rewrite
        ev.record()
        self.inflight.append((buf, ev, self.pending))
        self.pending = []

    def _pop(self, block):
        buf, ev, entries = self.inflight[0]
        if not ev.query():
            if not block:
                return False
            ev.synchronize()
        self.inflight.popleft()
        rows = buf.tolist()
        for slot, i_iter, extra in entries:
            self.emit(i_iter, rows[slot], extra)
        self.free.append((buf, ev))
        return True

    def poll(self):
        while self.inflight and self._pop(block=False):
            pass

    def drain(self):
        self.flush()
        while self.inflight:
            self._pop(block=True)

    def emit_now(self, i_iter, vals, extra=None):
        self.drain()
        self.emit(i_iter, vals, extra)


def _opt_hyper(opts):
    """The hyperparameters a captured optimizer step bakes in, per group."""
    def f(v):
        return float(v.item()) if torch.is_tensor(v) else float(v)
    return tuple((f(g["lr"]), tuple(f(b) for b in g.get("betas", ())), f(g.get("eps", 0.0)),
                  f(g.get("weight_decay", 0.0))) for o in opts for g in o.param_groups)


def _detached_snapshot(state):
    """Copies of the tensors a capture's warm-up changes.  Detached, under
    no_grad: a clone of a parameter made with grad mode on would hold its
    AccumulateGrad node (created on the launching stream) alive into the
    capture, where it then runs on the wrong stream (the HIP runtime crashed
    at capture end).  Checked, so a future state list cannot bring it back."""
    with torch.no_grad():
        saved = [t.detach().clone() for t in state]
    bad = [i for i, t in enumerate(saved) if t.grad_fn is not None or t.requires_grad]
    if bad:
        raise RuntimeError(f"capture state snapshot {bad} carries autograd history")
    return saved


class _GraphedIteration:
    """One training iteration fed by DeviceCloudLoaders as ONE HIP graph: each
    loader's batch gathered (+ device jitter) into static input buffers from a
    static copy of its epoch order at a device batch cursor
    (pcadv_gather_clouds_at), the fused step, then pcadv_iter_epilogue
    (loaders' RNG steps and cursors += 1, losses into the loss ring).  Per
    iteration the host only replays; at an epoch start it rewrites the order
    (the loader's own epoch_order(): the draws iterating it would make) and
    zeroes the cursor.  Ragged batches (drop_last=False) are gathered eagerly
    from the same order, their cursors advanced alike.  Graphs per `semi`
    flag, captured on first use; the capture's warm-up leaves parameters, Adam
    state, counters and the ring as they were."""

    def __init__(self, step, loaders, ring, optimizers=()):
        self.step, self.loaders, self.ring = step, loaders, ring
        # a capture bakes the optimizers' Python-float hyperparameters (lr,
        # betas, eps) into its kernels: a change (a scheduler, the reference's
        # adjust_learning_rate) drops the graphs and recaptures
        self.optimizers = tuple(o for o in optimizers if o is not None)
        self._hyper = _opt_hyper(self.optimizers)
        B, N, dev = step.B, step.N, step.device
        L = len(loaders)
        self.B, self.L = B, L
        self.counters = torch.zeros(2 * L, dtype=torch.int32, device=dev)  # RNG steps | cursors
        for k, ld in enumerate(loaders):
            self.counters[k:k + 1].copy_(ld.step)
            ld.step = self.counters[k:k + 1]  # the loader keeps using it (eager gathers too)
        self.order = [torch.zeros(ld.order_len, dtype=torch.int64, device=dev) for ld in loaders]
        self.pos = [None] * L  # host: next batch of the current epoch
        self.pts = [torch.zeros(B, N, 3, device=dev) for _ in loaders]
        # the labelled split's label width (the gather writes B x width int64)
        lw = max([int(ld.labels.shape[1]) for ld in loaders if ld.labels is not None] or [1])
        self.lab = torch.zeros(B, lw, dtype=torch.int64, device=dev)
        self.graphs = {}

    def next_batches(self):
        """Advance every loader by one batch: [(batch index k, size)]."""
        out = []
        for k, ld in enumerate(self.loaders):
            if self.pos[k] is None or self.pos[k] >= len(ld):
                self.order[k].copy_(ld.epoch_order())
                self.counters[self.L + k:self.L + k + 1].zero_()
                self.pos[k] = 0
            kk = self.pos[k]
            self.pos[k] += 1
            out.append((kk, min(ld.B, ld.order_len - kk * ld.B)))
        return out

    def eager_batches(self, batches):
        """Gather this iteration's batches eagerly (a ragged one among them):
        the loaders' own gather (RNG step advanced there), cursors += 1."""
        outs = []
        for k, (ld, (kk, size)) in enumerate(zip(self.loaders, batches)):
            idx = self.order[k][kk * ld.B:kk * ld.B + size].contiguous()
            outs.append(ld.gather(idx, _checked=True))
        self.counters[self.L:] += 1
        return outs

    def _gathers(self):
        """Every loader's batch at its device cursor: one launch for all of
        them (dataset.gather_at_multi)."""
        L = self.L
        items = [(ld, self.order[k], self.counters[L + k:L + k + 1], self.pts[k],
                  self.lab if (k == 0 and ld.labels is not None) else None, None)
                 for k, ld in enumerate(self.loaders)]
        if len(items) == 1:
            ld, *rest = items[0]
            ld.gather_at(*rest)
        else:
            gather_at_multi(items)

    def _gather_jobs(self):
        L = self.L
        return [ld._gather_job(self.order[k], self.counters[L + k:L + k + 1], self.pts[k],
                               self.lab if (k == 0 and ld.labels is not None) else None)
                for k, ld in enumerate(self.loaders)]

    def _folded(self):
        """The fused steps gather their batches in their first launch and run
        the iteration epilogue in their last: the graph is the step's launches
        alone."""
        st = self.step
        if not hasattr(st, "folded_gather") or self.lab.shape[1] != 1:
            return None
        stack = contextlib.ExitStack()
        stack.enter_context(st.folded_gather(self._gather_jobs()))
        stack.enter_context(st.folded_epilogue(self.counters, 2 * self.L, self.ring))
        return stack

    def _body(self, semi):
        L = self.L
        fold = self._folded()
        if fold is None:
            self._gathers()
        with (fold or contextlib.nullcontext()):
            if L == 2:
                self.step(self.pts[0], self.lab[:, 0], self.pts[1], semi=semi)
            else:
                self.step(self.pts[0], self.lab[:, 0])
        if fold is None:
            self.ring.write(self.step.losses, self.counters, 2 * L)

    def _graph(self, semi):
        g = self.graphs.get(semi)
        if g is None:
            st = self.step
            state = self._state()
            saved = _detached_snapshot(state)
            cur = torch.cuda.current_stream()
            side = torch.cuda.Stream(device=st.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):  # warm-up outside the capture
                self._body(semi)
            cur.wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._body(semi)
            torch.cuda.synchronize()
            with torch.no_grad():
                for dst, src in zip(state, saved):
                    dst.copy_(src)
            if hasattr(st, "after_capture"):
                st.after_capture()
            self.graphs[semi] = g
        return g

    def _check_hyper(self):
        h = _opt_hyper(self.optimizers)
        if h != self._hyper:
            self.graphs.clear()
            if hasattr(self.step, "sync_hyper"):
                self.step.sync_hyper()
            self._hyper = h

    def replay(self, semi=False):
        self._check_hyper()
        self._graph(semi).replay()
        return self.step.losses

    def _state(self):
        st = self.step
        if hasattr(st, "graph_state"):  # a step that names its own state
            pre = st.graph_state()
        else:
            pre = [t for t in (getattr(st, n, None) for n in
                               ("g_param", "g_m", "g_v", "d_param", "d_m", "d_v", "step_count"))
                   if t is not None]
        return pre + [self.counters, self.ring.count, self.ring.ring]


class _DPIteration(_GraphedIteration):
    """_GraphedIteration for a data-parallel rank (DeviceCloudLoaders sharded
    over the process group, AdvTrainStep keyed to this rank's global rows):
    [gathers + the whole step without Adam] | all-reduce(AVG) of the 4.2 MB
    G + D gradient buffer and of the loss vector | [both Adams + the iteration
    epilogue].  Over RCCL the collectives are captured with the rest: the
    iteration is ONE HIP graph (measured on a one-rank RCCL group, bench.py
    --config dp1: 11 us per iteration over the plain step, against 62 us for
    the round-5 form - four graphs around bucketed, overlapped host-issued
    all-reduces, whose overlap never materialised: the trace shows the
    feature backward waiting for the RCCL kernel).  Over gloo
    (CPU collectives, not capturable) two graphs around eager all-reduces.
    With equal shards the replicas take exactly the one-process step on the
    global batch (CE / BCE are batch means; the logged losses are the ranks'
    average, i.e. the global batch's)."""

    def __init__(self, step, loaders, ring, group=None, optimizers=()):
        super().__init__(step, loaders, ring, optimizers)
        self.group = group
        import torch.distributed as dist
        self.captured = dist.get_backend(group) == "nccl"

    def _part(self, k, semi):
        st, L = self.step, self.L
        if k == 1:
            if hasattr(st, "folded_gather"):
                with st.folded_gather(self._gather_jobs()):
                    st(self.pts[0], self.lab[:, 0], self.pts[1], apply_adam=False, semi=semi)
            else:
                self._gathers()
                st(self.pts[0], self.lab[:, 0], self.pts[1], apply_adam=False, semi=semi)
        else:
            st.adam()
            self.ring.write(st.losses, self.counters, 2 * L)

    def _average(self):
        from .distributed import _avg_async
        done = _avg_async(self.step.grad_flat, self.group)
        done_loss = _avg_async(self.step.losses, self.group)
        done()
        done_loss()

    def _whole(self, semi):
        self._part(1, semi)
        self._average()
        self._part(2, semi)

    def _graph(self, semi):
        gs = self.graphs.get(semi)
        if gs is None:
            state = self._state()
            saved = _detached_snapshot(state)
            cur = torch.cuda.current_stream()
            side = torch.cuda.Stream(device=self.step.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):  # warm-up outside the capture (every rank alike)
                self._whole(semi)
            cur.wait_stream(side)
            torch.cuda.synchronize()
            if self.captured:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self._whole(semi)
                gs = [g]
            else:
                gs = []
                for k in (1, 2):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        self._part(k, semi)
                    gs.append(g)
            torch.cuda.synchronize()
            with torch.no_grad():
                for dst, src in zip(state, saved):
                    dst.copy_(src)
            self.graphs[semi] = gs
        return gs

    def replay(self, semi=False):
        self._check_hyper()
        gs = self._graph(semi)
        if len(gs) == 1:
            gs[0].replay()
        else:
            gs[0].replay()
            self._average()
            gs[1].replay()
        return self.step.losses


class _SegGraphedIteration(_GraphedIteration):
    """run_training_pointnet_seg's iteration fed by a ShapeNet DeviceCloudLoader
    as ONE HIP graph: the batch gather (points, class ids, part ids, device
    jitter) at the device cursor, the one-hot class vector built on the device,
    SegTrainStep (forward, per-point CE, backward, Adam), and the iteration
    epilogue (counters += 1, the loss into the ring)."""

    def __init__(self, step, loader, ring, optimizers=()):
        step.B, step.N = loader.B, loader.npts  # the static batch shape
        super().__init__(step, (loader,), ring, optimizers)
        dev = step.device
        self.seg = torch.zeros(loader.B, loader.npts, dtype=torch.int64, device=dev)
        self.oh = torch.zeros(loader.B, 1, loader.ds.num_classes, device=dev)

    def _body(self, semi):
        ld = self.loaders[0]
        ld.gather_at(self.order[0], self.counters[1:2], self.pts[0], self.lab, out_seg=self.seg)
        self.oh.zero_()
        self.oh.scatter_(2, self.lab[:, :1].unsqueeze(1), 1.0)  # one_hot (shapeNetData.py)
        self.step(self.pts[0], self.oh, self.seg)
        self.ring.write(self.step.loss.view(1), self.counters, 2)


def _dp_world(*loaders):
    """World size of data-parallel (sharded) DeviceCloudLoaders, 1 if none;
    every loader must agree."""
    ws = {int(getattr(l, "world", 1)) for l in loaders}
    if len(ws) != 1:
        raise ValueError(f"loaders sharded over different world sizes {sorted(ws)}")
    return ws.pop()


class _AutogradStep:
    """A trainer body run through torch's autograd and the user's optimizers, as
    a step _GraphedIteration can capture (the layer-by-layer kernels; every
    optimizer must be capturable, e.g. torch.optim.Adam(capturable=True)).
    Subclasses set self.opts and self.losses (a static device tensor).

    The body starts with zero_grad(set_to_none=True), as the reference's does:
    inside the capture each backward then takes its gradient tensor as p.grad
    (allocated once, from the graph's pool) instead of adding it into a zeroed
    one, which would replay one add kernel per parameter (28 of them, about
    0.11 ms of the feature-transform cls step)."""

    def _params(self):
        return [p for o in self.opts for g in o.param_groups for p in g["params"]]

    def graph_state(self):
        """Parameters, existing gradients and optimizer state: restored after
        the capture's warm-up.  Optimizer state the warm-up creates (a first
        step) is reset to its fresh zeros by after_capture()."""
        params = self._params()
        self._fresh = [p for o in self.opts for g in o.param_groups for p in g["params"]
                       if p not in o.state or not o.state[p]]
        ts = list(params) + [p.grad for p in params if p.grad is not None]
        for o in self.opts:
            for p in (q for g in o.param_groups for q in g["params"]):
                if p in o.state:
                    ts += [v for v in o.state[p].values() if torch.is_tensor(v)]
        return ts

    def after_capture(self):
        for o in self.opts:
            for p in self._fresh:
                for v in o.state.get(p, {}).values():
                    if torch.is_tensor(v):
                        v.zero_()
        # the graph reads and writes these gradient buffers: kept alive here
        # (every captured graph's) and rebound after an eager iteration
        self._grads = [(p, p.grad) for p in self._params() if p.grad is not None]
        self._kept = getattr(self, "_kept", []) + [self._grads]

    def rebind_grads(self):
        """After an eager iteration (zero_grad(set_to_none=True) gave p.grad new
        tensors): its gradients into the captured buffers, rebound as p.grad."""
        for p, g in getattr(self, "_grads", ()):
            if p.grad is None:
                g.zero_()
            elif p.grad is not g:
                g.copy_(p.grad)
            p.grad = g

    @staticmethod
    def _capturable(args, optimizers):
        return (bool(getattr(args, "use_graph", True))
                and str(args.device).split(":")[0] == "cuda"
                and all(g.get("capturable", False) for o in optimizers for g in o.param_groups))


class _AutogradClsStep(_AutogradStep):
    """run_training_pointnet_cls's autograd body (utils/trainer.py:254-268:
    CE (x lambda_cls) + lambda_regu x the feature-transform regulariser,
    backward, optimizer.step()).  losses = [loss_cls, loss_regu]."""

    def __init__(self, model, optimizer, cls_loss, lambda_cls, lambda_regu, B, N, device):
        self.model, self.opt, self.cls_loss = model, optimizer, cls_loss
        self.opts = (optimizer,)
        self.lambda_cls, self.lambda_regu = lambda_cls, lambda_regu
        self.B, self.N, self.device = B, N, torch.device(device)
        self.losses = torch.zeros(2, device=self.device)
        self._fresh = []

    def __call__(self, pts, lab):
        self.opt.zero_grad()  # see _AutogradStep: no accumulate kernels in the graph
        pred, _, high_feat = self.model(pts)
        l = self.cls_loss(pred, lab)
        l_regu = feature_transform_regularizer(high_feat)
        loss = self.lambda_cls * l + self.lambda_regu * l_regu
        loss.backward()
        self.opt.step()
        self.losses[0].copy_(l.detach())
        self.losses[1].copy_(l_regu.detach())

    @staticmethod
    def graphable(model, optimizer, args, loader):
        return (isinstance(model, PointNetCls) and model.feature_transform
                and _device_loaders(loader) and _AutogradStep._capturable(args, (optimizer,)))


def _adv_body(model, model_D, optimizer, optimizer_D, gan_loss, cls_loss, pts, cls, pts_nogt,
              pool_gt, pool_nogt, args, semi_loss=None, semi_on=False, set_to_none=True):
    """run_training's iteration body through autograd (utils/trainer.py:449-559,
    the semi term :716-743): returns the device losses (loss_cls, loss_adv,
    loss_D_gt, loss_D_nogt) and the semi loss as a float (0.0 when off)."""
    gt_label, nogt_label = 1, 0
    optimizer.zero_grad(set_to_none=set_to_none)
    optimizer_D.zero_grad(set_to_none=set_to_none)
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
    D_out = model_D(pool_gt.query(pred_gt_softmax.detach()))
    loss_D1 = gan_loss(D_out, make_D_label(D_out, gt_label, args.device, random=True)) * 0.5
    loss_D1.backward()
    D_out = model_D(pool_nogt.query(pred_nogt_softmax.detach()))
    loss_D2 = gan_loss(D_out, make_D_label(D_out, nogt_label, args.device, random=True)) * 0.5
    loss_D2.backward()
    optimizer.step()
    optimizer_D.step()
    return l, loss_adv, loss_D1, loss_D2, loss_semi_value


class _AutogradAdvStep(_AutogradStep):
    """run_training's autograd body (_adv_body, without the semi term, whose
    ignore test reads the host) for configurations off the fused step (e.g. a
    feature-transform generator, other optimizers or losses).  losses =
    [loss_cls, loss_adv, loss_D_gt, loss_D_nogt, 0, 0]."""

    def __init__(self, model, model_D, optimizer, optimizer_D, gan_loss, cls_loss, pools, args,
                 B, N):
        self.parts = (model, model_D, optimizer, optimizer_D, gan_loss, cls_loss)
        self.pools, self.args = pools, args
        self.opts = (optimizer, optimizer_D)
        self.B, self.N, self.device = B, N, torch.device(args.device)
        self.losses = torch.zeros(6, device=self.device)
        self._fresh = []

    def __call__(self, pts, lab, pts_nogt, semi=False):
        if semi:
            raise ValueError("_AutogradAdvStep: the semi term is not capturable")
        out = _adv_body(*self.parts, pts, lab, pts_nogt, *self.pools, self.args)
        self.losses[:4].copy_(torch.stack([t.detach() for t in out[:4]]))

    @staticmethod
    def graphable(optimizer, optimizer_D, pools, args, loaders):
        return (all(p.pool_size == 0 for p in pools) and _device_loaders(*loaders)
                and loaders[0].B == loaders[1].B and loaders[0].npts == loaders[1].npts
                and _AutogradStep._capturable(args, (optimizer, optimizer_D)))


def _device_loaders(*loaders):
    from .dataset import DeviceCloudLoader
    return all(isinstance(l, DeviceCloudLoader) and l.kind in ("modelnet_gt", "modelnet_nogt")
               for l in loaders)


def _fusable(model, model_D, optimizer, optimizer_D, gan_loss, cls_loss, args):
    """The configuration the fused steps implement: False, or the step class
    (AdvTrainStep; AdvFtTrainStep for a feature-transform generator unless
    args.fused_ft is False)."""
    if not (isinstance(model, PointNetCls) and isinstance(model_D, DeepConvDiscNet)):
        return False
    if model.fc3.out_features != 40:
        return False
    if model.feature_transform and not getattr(args, "fused_ft", True):
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
    # the fused Adam applies one (betas, eps) pair to both networks (only the
    # learning rates are separate): a discriminator optimizer with its own
    # betas / eps runs the autograd body with the torch optimizers
    g, gd = optimizer.param_groups[0], optimizer_D.param_groups[0]
    if tuple(map(float, g["betas"])) != tuple(map(float, gd["betas"])) \
            or float(g["eps"]) != float(gd["eps"]):
        return False
    if type(gan_loss) is not torch.nn.BCEWithLogitsLoss or gan_loss.weight is not None \
            or gan_loss.pos_weight is not None or gan_loss.reduction != "mean":
        return False
    if type(cls_loss) is not torch.nn.CrossEntropyLoss or cls_loss.weight is not None \
            or cls_loss.reduction != "mean" or cls_loss.label_smoothing != 0.0:
        return False
    return AdvFtTrainStep if model.feature_transform else AdvTrainStep


def _pooled_d_grads(step, model_D, gan_loss, pool_gt, pool_nogt, B, device):
    """The discriminator half of utils/trainer.py:521-556 with image pools: after
    a fused step ran without its Adam update (G's gradients, and its
    classification / adversarial / semi loss lines, do not see the pools), D's
    gradient is replaced by the reference's two backward passes on
    pool.query(log_softmax(logits)) of this iteration's GT and no-GT logits,
    accumulated into the flat gradient buffer the fused Adam reads (the D
    parameters' .grad are views of it), and the D loss lines follow."""
    logp = F.log_softmax(step.logits[:2 * B], dim=1)
    step.d_grad.zero_()
    d_out = model_D(pool_gt.query(logp[:B].detach()))
    loss_d1 = gan_loss(d_out, make_D_label(d_out, 1, device, random=True)) * 0.5
    loss_d1.backward()
    d_out = model_D(pool_nogt.query(logp[B:].detach()))
    loss_d2 = gan_loss(d_out, make_D_label(d_out, 0, device, random=True)) * 0.5
    loss_d2.backward()
    views = _views(step.d_grad, model_D, D_LAYOUT)
    for name, p in model_D.named_parameters():
        if p.grad is None or p.grad.data_ptr() != views[name].data_ptr():
            raise RuntimeError(f"D parameter {name}: .grad is no longer a view of the fused "
                               "step's gradient buffer")
    step.losses[2:4].copy_(torch.stack((loss_d1.detach(), loss_d2.detach())))


def _save(model, model_D, args, tag):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_rank() != 0:
        return  # data parallel: the replicas are identical, rank 0 writes
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
    run_training_semi (pseudo-label term from iteration semi_start + 1).

    Fast path: with the hot path's configuration (see _fusable) every
    iteration whose GT and no-GT batches have the same shape is one fused
    native step; when both loaders are DeviceCloudLoaders the batch gathers
    and the step replay as one HIP graph per iteration (args.use_graph, default
    on), fed by the loaders' own epoch orders.  Loss lines are read
    asynchronously (no host sync per iteration), every args.log_every
    iterations (default 1, as the reference logs every iteration).  A
    feature-transform generator runs AdvFtTrainStep (the point-wise kernels
    over both batches + the fused step's tail; args.fused_ft = False keeps the
    autograd body).  Off the fused steps (other optimizers or losses) the body
    runs through autograd (_adv_body); with capturable optimizers and
    DeviceCloudLoaders its full, semi-free iterations are HIP graphs too
    (_AutogradAdvStep)."""
    max_test_accu = float("-inf")
    max_train_epoch = 0
    fused = _fusable(model, model_D, optimizer, optimizer_D, gan_loss, cls_loss, args)
    if semi_loss is not None and not _semi_fusable(semi_loss):
        fused = False
    # ImagePool(pool_size > 0): the fused step's G half stands, D's gradient is
    # recomputed on the pools' outputs (_pooled_d_grads); the pools draw from
    # the host's `random`, so these iterations are not graphed
    pooled = fused and (history_pool_gt.pool_size > 0 or history_pool_nogt.pool_size > 0)
    step = None
    log_every = max(1, int(getattr(args, "log_every", 1)))
    graphed = (fused and not pooled and bool(getattr(args, "use_graph", True))
               and _device_loaders(trainloader_gt, trainloader_nogt)
               and trainloader_gt.B == trainloader_nogt.B
               and trainloader_gt.npts == trainloader_nogt.npts
               and trainloader_gt.B <= MAX_FUSED_B
               and (fused is not AdvFtTrainStep or trainloader_gt.npts % 128 == 0))
    # off the fused step, with capturable optimizers over DeviceCloudLoaders:
    # each full, semi-free iteration's gathers + autograd body as one HIP graph
    ag_graphed = (not fused) and _AutogradAdvStep.graphable(
        optimizer, optimizer_D, (history_pool_gt, history_pool_nogt), args,
        (trainloader_gt, trainloader_nogt))
    gi = None
    tb = getattr(args, "tensorboard", False) and writer is not None
    # data parallelism: DeviceCloudLoaders sharded over the process group
    # (DeviceCloudLoader(..., world_size=W)); every iteration is the fused step
    # on this rank's shard, graphed around the gradient all-reduces (_DPIteration)
    world = _dp_world(trainloader_gt, trainloader_nogt) if _device_loaders(
        trainloader_gt, trainloader_nogt) else 1
    rank = 0
    if world > 1:
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() != world:
            raise RuntimeError(f"loaders sharded over {world} ranks: initialise a process group of "
                               "that size first")
        if not graphed or fused is not AdvTrainStep:
            raise NotImplementedError(
                "data-parallel run_training runs the fused step graphed over DeviceCloudLoaders: "
                "PointNetCls(k=40) + DeepConvDiscNet(40, 1), Adam, CE / BCE, ImagePool(0), equal "
                "GT / no-GT batches (args.use_graph on)")
        if semi_loss is not None and args.semi_start > 0:
            # k_head_bwd normalises the pseudo-label CE by this rank's own kept
            # count (a data-dependent mean), so averaging the ranks' gradients
            # is not the global batch's mean over all kept clouds
            raise NotImplementedError(
                "data-parallel run_training_semi: the pseudo-label CE is a mean over each rank's "
                "kept clouds, which a gradient average does not turn into the global batch's "
                "mean; run the semi phase on one process")
        rank = dist.get_rank()

    def emit(i_iter, vals, semi_on):
        loss_D_value = vals[2] + vals[3]
        train_logger.info("iter = {0:8d}/{1:8d} loss_cls = {2:.3f} loss_adv = {3:.3f} "
                          "loss_D = {4:.3f}".format(i_iter, args.total_iterations, vals[0],
                                                    vals[1], loss_D_value))
        if tb:
            writer.add_scalar("Loss/train_cls", vals[0], i_iter)
            writer.add_scalar("Loss/train_adv", vals[1], i_iter)
            writer.add_scalar("Loss/train_disc", loss_D_value, i_iter)
            if semi_loss is not None:
                writer.add_scalar("Loss/train_semi", vals[4] if semi_on else 0.0, i_iter)

    log = _LossRing(emit, 6, args.device)
    if graphed or ag_graphed:  # the loaders' own epoch orders replace the (fresh) iterators given
        B0, N0 = trainloader_gt.B, trainloader_gt.npts

    def fused_step(B, N):
        nonlocal step
        if step is None or step.N != N or step.B < B:
            if step is not None:  # the replacement adopts the Adam state: count included
                step.sync_optimizer_state()
            step = fused(model, model_D, B, N,
                         optimizer=optimizer, optimizer_D=optimizer_D,
                         lambda_cls=args.lambda_cls, lambda_adv=args.lambda_adv,
                         seed=int(getattr(args, "seed", 0)) + i_iter,
                         device=args.device,
                         lambda_semi=float(getattr(args, "lambda_semi", 1.0)),
                         semi_th=float(getattr(args, "semi_TH", 0.8)),
                         rng_rank=rank, rng_world=world)
            if world > 1:  # identical replicas: rank 0's parameters and seed
                from .distributed import DataParallelAdvStep
                DataParallelAdvStep(step, broadcast_params=True)
        step.sync_hyper()  # lr / betas / eps as the optimizers hold them now
        return step

    for i_iter in range(args.total_iterations):
        # trainer.py:432-433; inside this loop only run_testing changes the modes
        # (model.eval()), so the recursive train() is re-applied only then
        if i_iter == 0 or not model.training:
            model.train()
        if i_iter == 0 or not model_D.training:
            model_D.train()
        semi_on = semi_loss is not None and args.semi_start > 0 and i_iter > args.semi_start
        losses = None
        if graphed or ag_graphed:
            if gi is None:
                gstep = (fused_step(B0, N0) if graphed else _AutogradAdvStep(
                    model, model_D, optimizer, optimizer_D, gan_loss, cls_loss,
                    (history_pool_gt, history_pool_nogt), args, B0, N0))
                gi = (_DPIteration(gstep, (trainloader_gt, trainloader_nogt), log,
                                   optimizers=(optimizer, optimizer_D)) if world > 1
                      else _GraphedIteration(gstep, (trainloader_gt, trainloader_nogt), log,
                                             optimizers=(optimizer, optimizer_D)))
            bt = gi.next_batches()
            if all(size == B0 for _, size in bt) and not (ag_graphed and semi_on):
                losses = gi.replay(semi=semi_on)
            else:  # a ragged last batch: gathered eagerly from the same epoch order
                (pts, cls), pts_nogt = gi.eager_batches(bt)
        else:
            batch, trainloader_gt_iter = _next(trainloader_gt, trainloader_gt_iter)
            pts, cls = batch
            pts_nogt, targetloader_nogt_iter = _next(trainloader_nogt, targetloader_nogt_iter)
        if losses is None:
            pts = pts.float().to(args.device).contiguous()
            cls = cls.long().to(args.device).contiguous()
            pts_nogt = pts_nogt.float().to(args.device).contiguous()
            if (fused and pts.shape == pts_nogt.shape and pts.shape[0] <= MAX_FUSED_B
                    and (fused is not AdvFtTrainStep or pts.shape[1] % 128 == 0)):
                st = fused_step(pts.shape[0], pts.shape[1])
                if pooled:
                    losses = st(pts, cls, pts_nogt, apply_adam=False, semi=semi_on)
                    _pooled_d_grads(st, model_D, gan_loss, history_pool_gt, history_pool_nogt,
                                    pts.shape[0], args.device)
                    st.adam()
                else:
                    losses = st(pts, cls, pts_nogt, semi=semi_on)
                log.write(losses)

        if losses is not None:
            log.record(i_iter, semi_on, log=i_iter % log_every == 0)
        else:
            # off the fused step, or unequal GT / no-GT batches (a loader's
            # ragged last batch): the reference's body through autograd over the
            # same kernels; the torch optimizers continue from the fused step's
            # Adam state (moments are shared views, the step count is synced in
            # and out) or from the graphed body's (its gradient buffers rebound)
            if step is not None:
                step.sync_optimizer_state()
            l, loss_adv, loss_D1, loss_D2, loss_semi_value = _adv_body(
                model, model_D, optimizer, optimizer_D, gan_loss, cls_loss, pts, cls, pts_nogt,
                history_pool_gt, history_pool_nogt, args, semi_loss, semi_on)
            if step is not None:
                step.after_torch_step()
            if gi is not None and ag_graphed:
                gi.step.rebind_grads()
            if i_iter % log_every == 0:
                log.emit_now(i_iter, [l.item(), loss_adv.item(), loss_D1.item(), loss_D2.item(),
                                      loss_semi_value], semi_on)

        if i_iter % args.iter_save_epoch == 0:
            log.drain()
            if step is not None:
                step.sync_optimizer_state()
            if semi_loss is None:
                tag = i_iter // args.iter_save_epoch
            else:  # trainer.py:789
                tag = int(round(i_iter / len(trainloader_gt)))
            _save(model, model_D, args, "train_epoch_{}".format(tag))
        if i_iter % args.iter_test_epoch == 0:
            log.drain()
            curr_accu, _ = run_testing(testloader, model, cls_loss, test_logger, i_iter, writer, args)
            if max_test_accu < curr_accu:
                max_test_accu = curr_accu
                max_train_epoch = i_iter // args.iter_test_epoch
                _save(model, model_D, args, "train_best")

    log.drain()
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
    PointNetCls(k=40), CrossEntropyLoss and Adam on the HIP device each
    iteration is one ClsTrainStep (pcadv_cls_step), or with
    feature_transform=True one ClsFtTrainStep (its regulariser in the loss);
    otherwise the reference's body runs through autograd over the same
    kernels."""
    from .step import ClsFtTrainStep, ClsTrainStep
    max_test_accu = float("-inf")
    max_train_epoch = 0
    fusable = (isinstance(model, PointNetCls)
               and model.fc3.out_features == 40 and type(optimizer) is torch.optim.Adam
               and len(optimizer.param_groups) == 1
               and not optimizer.param_groups[0].get("weight_decay", 0)
               and not optimizer.param_groups[0].get("amsgrad")
               and type(cls_loss) is torch.nn.CrossEntropyLoss and cls_loss.weight is None
               and cls_loss.reduction == "mean" and cls_loss.label_smoothing == 0.0
               and str(args.device).split(":")[0] == "cuda")
    fused = fusable and not model.feature_transform
    # feature_transform=True: the fused FT cls step (step.ClsFtTrainStep: the
    # regulariser joins the loss there); args.fused_ft = False keeps the
    # autograd body
    fused_ft = fusable and model.feature_transform and bool(getattr(args, "fused_ft", True))
    step = None
    graphed = ((fused or fused_ft) and bool(getattr(args, "use_graph", True))
               and _device_loaders(trainloader_gt) and trainloader_gt.B <= MAX_FUSED_B
               and (not fused_ft or trainloader_gt.npts % 128 == 0))
    gi = None
    log_every = max(1, int(getattr(args, "log_every", 1)))
    # feature_transform=True off the fused step, with a capturable optimizer over
    # a DeviceCloudLoader: each full batch's gather + autograd body replayed as
    # one HIP graph
    ft_graphed = (not fused and not fused_ft) and _AutogradClsStep.graphable(
        model, optimizer, args, trainloader_gt)

    def emit(i_iter, vals, regu):
        train_logger.info("iter = {0:8d}/{1:8d} loss_cls = {2:.3f} loss regu = {3:.3f} ".format(
            i_iter, args.total_iterations, vals[0], vals[1] if regu is None else regu))

    two = ft_graphed or fused_ft  # [loss_cls, loss_regu] in the ring
    log = _LossRing(emit, 2 if two else 1, args.device)

    def fused_step(B, N):
        nonlocal step
        if step is None or step.N != N or step.B < B:
            if step is not None:
                step.sync_optimizer_state()
            seed = int(getattr(args, "seed", 0)) + i_iter
            step = (ClsFtTrainStep(model, B, N, optimizer=optimizer, lambda_cls=args.lambda_cls,
                                   lambda_regu=args.lambda_regu, seed=seed, device=args.device)
                    if fused_ft else
                    ClsTrainStep(model, B, N, optimizer=optimizer, lambda_cls=args.lambda_cls,
                                 seed=seed, device=args.device))
        step.sync_hyper()
        return step

    for i_iter in range(args.total_iterations):
        if i_iter == 0 or not model.training:  # only run_testing's eval() changes it here
            model.train()
        l_regu = None
        losses = None
        if graphed or ft_graphed:
            if gi is None:
                gstep = (fused_step(trainloader_gt.B, trainloader_gt.npts) if graphed else
                         _AutogradClsStep(model, optimizer, cls_loss, args.lambda_cls,
                                          args.lambda_regu, trainloader_gt.B,
                                          trainloader_gt.npts, args.device))
                gi = _GraphedIteration(gstep, (trainloader_gt,), log, optimizers=(optimizer,))
            bt = gi.next_batches()
            if bt[0][1] == trainloader_gt.B:
                losses = gi.replay()
            else:
                (pts, cls), = gi.eager_batches(bt)
        else:
            batch, trainloader_gt_iter = _next(trainloader_gt, trainloader_gt_iter)
            pts, cls = batch
        if losses is None:
            pts, cls = pts.float().to(args.device).contiguous(), cls.long().to(args.device).contiguous()
            if ((fused or fused_ft) and pts.shape[0] <= MAX_FUSED_B
                    and (not fused_ft or pts.shape[1] % 128 == 0)):
                losses = fused_step(pts.shape[0], pts.shape[1])(pts, cls)
                log.write(losses)
        if losses is not None:
            log.record(i_iter, None if two else 0.0, log=i_iter % log_every == 0)
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
            if gi is not None and ft_graphed:
                gi.step.rebind_grads()
            if i_iter % log_every == 0:
                log.emit_now(i_iter, [l.item()], 0.0 if l_regu is None else l_regu.item())
        if i_iter % args.iter_save_epoch == 0:
            log.drain()
            if step is not None:
                step.sync_optimizer_state()
            torch.save(model.state_dict(), os.path.join(
                args.exp_dir, "model_train_epoch_{}.pth".format(i_iter // len(trainloader_gt))))
        if i_iter % args.iter_test_epoch == 0:
            log.drain()
            curr_accu, _ = run_testing(testloader, model, cls_loss, test_logger, i_iter, writer, args)
            if max_test_accu < curr_accu:
                max_test_accu = curr_accu
                max_train_epoch = i_iter // args.iter_test_epoch
                torch.save(model.state_dict(), os.path.join(args.exp_dir, "model_train_best.pth"))
    log.drain()
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
    from .dataset import DeviceCloudLoader
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
    # fast path: a ShapeNet DeviceCloudLoader (the split resident in HBM) runs
    # every full batch as one HIP graph (_SegGraphedIteration); the loss lines
    # are read from the device ring asynchronously (no host sync per iteration)
    graphed = (fused and bool(getattr(args, "use_graph", True))
               and isinstance(trainloader_gt, DeviceCloudLoader)
               and trainloader_gt.kind == "shapenet_gt")
    gi = None
    log_every = max(1, int(getattr(args, "log_every", 1)))
    tb = getattr(args, "tensorboard", False) and writer is not None

    def emit(i_iter, vals, extra):
        train_logger.info("iter = {0:8d}/{1:8d} loss_seg = {2:.3f} ".format(
            i_iter, args.total_iterations, vals[0]))
        if tb:
            writer.add_scalar("Loss/train_seg", vals[0], i_iter)

    log = _LossRing(emit, 1, args.device)

    def fused_step():
        nonlocal step
        if step is None:
            step = SegTrainStep(model, optimizer=optimizer, lambda_seg=args.lambda_seg,
                                device=args.device)
        step.sync_hyper()
        return step

    for i_iter in range(args.total_iterations):
        if i_iter == 0 or not model.training:  # only run_testing_seg's eval() changes it here
            model.train()
        loss = None
        if graphed:
            if gi is None:
                gi = _SegGraphedIteration(fused_step(), trainloader_gt, log, optimizers=(optimizer,))
            bt = gi.next_batches()
            if bt[0][1] == trainloader_gt.B:
                loss = gi.replay()
                fused_step()  # the eager step's hyperparameters follow the optimizer too
            else:  # a ragged last batch, gathered eagerly from the same epoch order
                (pts, cls, seg), = gi.eager_batches(bt)
        else:
            batch, trainloader_gt_iter = _next(trainloader_gt, trainloader_gt_iter)
            pts, cls, seg = batch
        if loss is None:
            pts = pts.float().to(args.device).contiguous()
            cls = cls.float().to(args.device).contiguous()
            seg = seg.long().to(args.device).contiguous()
            if fused:
                loss = fused_step()(pts, cls, seg)
                log.write(loss.view(1))
        if loss is not None:
            log.record(i_iter, None, log=i_iter % log_every == 0)
        else:
            optimizer.zero_grad()
            pred, global_gt = model(pts, cls)
            l = seg_loss(pred, seg)
            (args.lambda_seg * l).backward()
            optimizer.step()
            if i_iter % log_every == 0:
                log.emit_now(i_iter, [l.item()])
        if i_iter % args.iter_save_epoch == 0:
            log.drain()
            if step is not None:
                step.sync_optimizer_state()
            torch.save(model.state_dict(), os.path.join(
                args.exp_dir, "model_train_epoch_{}.pth".format(i_iter // len(trainloader_gt))))
        if i_iter % args.iter_test_epoch == 0:
            log.drain()
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
    log.drain()
    if step is not None:
        step.sync_optimizer_state()
    if getattr(args, "tensorboard", False) and writer is not None:
        writer.close()
    train_logger.info("=========================")
    train_logger.info("Max test accuracy: {:.4f}, at epoch: {}".format(max_test_accu, max_train_epoch))
    train_logger.info("Max cat mIoU: {:.4f}, at epoch: {}".format(max_test_cat_iou, max_train_cat_epoch))
    train_logger.info("Max all mIoU: {:.4f}, at epoch: {}".format(max_test_all_iou, max_train_all_epoch))
    return max_test_accu, max_test_cat_iou, max_test_all_iou
