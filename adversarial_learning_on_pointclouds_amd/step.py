"""The fused adversarial train step (one iteration of utils/trainer.py:run_training,
:426-559) as a single native call, optionally captured into a HIP graph.

Parameters of both networks are moved into one flat fp32 buffer each (state_dict
order, offsets = include/pcadv.h); the modules' Parameters become views of it,
so checkpoints, eval passes and torch optimizers keep working on the same
memory.  Both networks' gradients share ONE flat buffer (generator first), so a
data-parallel run averages them with a single all-reduce.  Adam moments are
flat too and are handed to a torch Adam optimizer's state as views
(exp_avg / exp_avg_sq), so optimizer.state_dict() stays meaningful.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch

from . import _lib
from ._lib import AdvArgs, D_LAYOUT, D_NUMEL, G_LAYOUT, G_NUMEL, check, stream_ptr

D_GRAD_OFFSET = (G_NUMEL + 63) // 64 * 64  # D grads start 256-B aligned
G_LATE_END = G_LAYOUT["fc1.weight"]  # grad_flat[:G_LATE_END]: the feature backward's (part 2)


def flatten_params(module, layout, numel, device):
    """Copy a module's parameters into one flat buffer and rebind them as views."""
    flat = torch.zeros(numel, device=device, dtype=torch.float32)
    named = dict(module.named_parameters())
    if set(named) != set(layout):
        raise ValueError(f"{type(module).__name__}: parameters {sorted(set(named) ^ set(layout))} "
                         "do not match the fused-step layout")
    for name, off in layout.items():
        p = named[name]
        n = p.numel()
        flat[off:off + n].copy_(p.detach().reshape(-1))
        p.data = flat[off:off + n].view_as(p)
    return flat


def _views(flat, module, layout):
    named = dict(module.named_parameters())
    return {name: flat[off:off + named[name].numel()].view_as(named[name])
            for name, off in layout.items()}


def _precision(name):
    """Feature-forward precision code of pcadv_adv_args.precision."""
    codes = {"fp32": 0, "bf16": 1}
    if name not in codes:
        raise ValueError(f"precision {name!r}: one of {sorted(codes)}")
    return codes[name]


# the feature-transform step's point-wise forward as two chained launches
# (pcadv_pw_chain, bitwise the per-layer pcadv_pw_fwd launches); PCADV_FT_CHAIN=0
# keeps the six per-layer launches (A/B)
_FT_CHAIN = os.environ.get("PCADV_FT_CHAIN", "1") == "1"


def _align(nbytes):
    return (nbytes + 255) // 256 * 256


def _adopt_adam_state(optimizer, module, m_flat, v_flat, layout):
    """Seed flat Adam moments from state an optimizer already holds (a
    load_state_dict before the first iteration, or the views of a previous
    step object the trainer rebuilt): exp_avg / exp_avg_sq are copied in and
    the largest 'step' is returned (0 when there is none)."""
    if optimizer is None:
        return 0
    steps = 0
    named = dict(module.named_parameters())
    for name, off in layout.items():
        st = optimizer.state.get(named[name])
        if not st or "exp_avg" not in st:
            continue
        n = named[name].numel()
        m_flat[off:off + n].copy_(st["exp_avg"].detach().reshape(-1))
        v_flat[off:off + n].copy_(st["exp_avg_sq"].detach().reshape(-1))
        steps = max(steps, int(float(st.get("step", 0))))
    return steps


def _step_tensor(optimizer, p, t):
    """'step' as torch.optim.Adam keeps it for p: an f32 scalar on p's device
    when its group is capturable or fused (the step then runs on the device,
    and Adam refuses a CPU count), a CPU f32 scalar otherwise."""
    for g in optimizer.param_groups:
        if any(q is p for q in g["params"]):
            if g.get("capturable", False) or g.get("fused", False):
                return torch.tensor(float(t), dtype=torch.float32, device=p.device)
            break
    return torch.tensor(float(t), dtype=torch.float32)


def set_optimizer_step(optimizer, t):
    """Every state entry's 'step' = t (the device step counter's value)."""
    if optimizer is None:
        return
    for p, st in optimizer.state.items():
        if st:
            st["step"] = _step_tensor(optimizer, p, t)


def _bind_adam_state(optimizer, module, m_flat, v_flat, grad_flat, layout, step_t):
    """p.grad and the optimizer's exp_avg / exp_avg_sq become views of the flat
    buffers; 'step' holds the completed-step count."""
    mv, vv, gv = _views(m_flat, module, layout), _views(v_flat, module, layout), \
        _views(grad_flat, module, layout)
    for name, p in module.named_parameters():
        p.grad = gv[name]
        if optimizer is not None:
            optimizer.state[p] = {"step": _step_tensor(optimizer, p, step_t),
                                  "exp_avg": mv[name], "exp_avg_sq": vv[name]}


def _fill_epilogue(a, epi, gather=None):
    """pcadv_adv_args.epi_* from (counters, ncounters, _LossRing) or None, and
    .gather / .ngather from a ctypes GatherJob array or None."""
    if gather is not None:
        a.gather, a.ngather = ctypes.addressof(gather), len(gather)
    if epi is None:
        return
    counters, n, ring = epi
    if n:
        a.epi_counters, a.epi_ncounters = counters.data_ptr(), n
    if ring is not None:
        a.epi_ring, a.epi_slots, a.epi_nl = ring.ring.data_ptr(), ring.slots, ring.nl
        a.epi_ring_count = ring.count.data_ptr()


class AdvTrainStep:
    """run_training's iteration body for PointNetCls(k=40) + DeepConvDiscNet(40, 1).

    Call with device tensors pts_gt (B, N, 3) f32, labels (B,) int64, pts_nogt
    (B, N, 3) f32.  Dropout masks and soft D labels are drawn on device from
    Philox keyed by (seed, step) unless given explicitly (parity mode:
    masks=(gt, nogt) each (B, 256) {0,1}; soft=(gt, nogt) each (B,)).
    Returns the device tensor [loss_cls, loss_adv, loss_D_gt, loss_D_nogt,
    loss_semi, semi_ratio] (no host sync: read it when you log,
    trainer.py:561-572).  semi=True adds run_training_semi's pseudo-label term
    (utils/trainer.py:716-743: lambda_semi x CrossEntropyLoss(ignore_index=255)
    of the no-GT logits against their argmax, clouds with D <= semi_th ignored).
    rng_rank / rng_world: this step is rank rng_rank of a data-parallel job of
    rng_world ranks, each holding the rows [rank B, rank B + B) of the global
    GT and no-GT batches: the device-drawn masks and labels are those of the
    one-process step on the global batch (pcadv_adv_args.rng_rank, ABI 6).
    """

    _epilogue = None  # (counters, ncounters, _LossRing) folded into the last launch
    _gather = None    # ctypes GatherJob array gathered by the first launch

    @contextlib.contextmanager
    def folded_epilogue(self, counters=None, ncounters=0, ring=None):
        """Within the block every step call also runs the training iteration's
        epilogue (counters[:ncounters] += 1, the losses into the loss ring; as
        pcadv_iter_epilogue) inside its own finishing launch - one launch less
        per graph-replayed iteration (pcadv_adv_args.epi_*)."""
        self._epilogue = (counters, int(ncounters), ring)
        try:
            yield
        finally:
            self._epilogue = None

    @contextlib.contextmanager
    def folded_gather(self, jobs):
        """Within the block every step call gathers its own input batches in
        its first launch (pcadv_adv_args.gather: the loaders' gather_at jobs,
        DeviceCloudLoader._gather_job, whose outputs are the step's inputs) -
        the iteration's gather launch disappears."""
        self._gather = (_lib.GatherJob * len(jobs))(*jobs)
        try:
            yield
        finally:
            self._gather = None

    def __init__(self, model, model_D, B, N, optimizer=None, optimizer_D=None, lr=1e-4,
                 lr_D=1e-4, betas=(0.9, 0.999), eps=1e-8, lambda_cls=1.0, lambda_adv=0.001,
                 seed=0, device="cuda", lambda_semi=1.0, semi_th=0.8, precision="fp32",
                 rng_rank=0, rng_world=1):
        self.lib = _lib.load()
        self.set_rng_rank(rng_rank, rng_world)
        self.model, self.model_D = model, model_D
        self.precision = _precision(precision)
        self.B, self.N = int(B), int(N)
        dev = torch.device(device)
        if dev.type != "cuda":
            raise ValueError("AdvTrainStep runs on the HIP device only")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        if optimizer is not None:
            g = optimizer.param_groups[0]
            lr, betas, eps = g["lr"], tuple(g["betas"]), g["eps"]
        if optimizer_D is not None:
            lr_D = optimizer_D.param_groups[0]["lr"]
        self.hp = dict(lr=float(lr), lr_D=float(lr_D), betas=betas, eps=float(eps),
                       lambda_cls=float(lambda_cls), lambda_adv=float(lambda_adv),
                       p=float(model.dropout.p), lambda_semi=float(lambda_semi),
                       semi_th=float(semi_th))
        self.g_param = flatten_params(model, G_LAYOUT, G_NUMEL, dev)
        self.d_param = flatten_params(model_D, D_LAYOUT, D_NUMEL, dev)
        self.grad_flat = torch.zeros(D_GRAD_OFFSET + D_NUMEL, device=dev)
        self.g_grad = self.grad_flat[:G_NUMEL]
        self.d_grad = self.grad_flat[D_GRAD_OFFSET:]
        self.g_m = torch.zeros_like(self.g_param)
        self.g_v = torch.zeros_like(self.g_param)
        self.d_m = torch.zeros_like(self.d_param)
        self.d_v = torch.zeros_like(self.d_param)
        # Adam state the optimizers already hold carries over (one step count
        # serves both networks: run_training steps them together)
        t0 = max(_adopt_adam_state(optimizer, model, self.g_m, self.g_v, G_LAYOUT),
                 _adopt_adam_state(optimizer_D, model_D, self.d_m, self.d_v, D_LAYOUT))
        self.step_count = torch.full((1,), t0, device=dev, dtype=torch.int32)
        self._bind = ((optimizer, model, self.g_m, self.g_v, self.g_grad, G_LAYOUT),
                      (optimizer_D, model_D, self.d_m, self.d_v, self.d_grad, D_LAYOUT))
        for args_ in self._bind:
            _bind_adam_state(*args_, t0)
        self.optimizers = (optimizer, optimizer_D)
        self.losses = torch.zeros(6, device=dev)
        self.logits = torch.zeros(2 * self.B, 40, device=dev)
        nbytes = self.lib.pcadv_adv_step_workspace_bytes(self.B, self.N)
        self.workspace = torch.empty(nbytes, device=dev, dtype=torch.uint8)
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.graph = None
        self._keep = []

    # ------------------------------------------------------------------
    def _args(self, pts_gt, labels, pts_nogt, masks, soft, apply_adam, semi=False, part=0):
        B, N = int(pts_gt.shape[0]), self.N
        if not 0 < B <= self.B:
            raise ValueError(f"batch of {B} clouds; this step was built for at most {self.B}")
        for t, nm, shape, dt in ((pts_gt, "pts_gt", (B, N, 3), torch.float32),
                                 (pts_nogt, "pts_nogt", (B, N, 3), torch.float32),
                                 (labels, "labels", (B,), torch.int64)):
            if (tuple(t.shape) != shape or t.dtype != dt or not t.is_contiguous()
                    or t.device != self.device):
                raise ValueError(f"{nm}: expected contiguous {dt} {shape} on {self.device}, "
                                 f"got {t.dtype} {tuple(t.shape)} on {t.device}")
        a = AdvArgs()
        a.B, a.N = B, N
        a.pts_gt, a.labels, a.pts_nogt = pts_gt.data_ptr(), labels.data_ptr(), pts_nogt.data_ptr()
        if masks is not None:
            for m in masks:
                if tuple(m.shape) != (B, 256) or m.dtype != torch.float32 or not m.is_contiguous():
                    raise ValueError("dropout masks must be contiguous float32 (B, 256)")
            a.drop_mask_gt, a.drop_mask_nogt = masks[0].data_ptr(), masks[1].data_ptr()
        if soft is not None:
            for s in soft:
                if s.numel() != B or s.dtype != torch.float32 or not s.is_contiguous():
                    raise ValueError("soft labels must be contiguous float32 with B elements")
            a.soft_gt, a.soft_nogt = soft[0].data_ptr(), soft[1].data_ptr()
        a.g_param, a.g_grad = self.g_param.data_ptr(), self.g_grad.data_ptr()
        a.g_m, a.g_v = self.g_m.data_ptr(), self.g_v.data_ptr()
        a.d_param, a.d_grad = self.d_param.data_ptr(), self.d_grad.data_ptr()
        a.d_m, a.d_v = self.d_m.data_ptr(), self.d_v.data_ptr()
        a.step_count = self.step_count.data_ptr()
        hp = self.hp
        a.lr_g, a.lr_d = hp["lr"], hp["lr_D"]
        a.beta1, a.beta2, a.eps = hp["betas"][0], hp["betas"][1], hp["eps"]
        a.lambda_cls, a.lambda_adv, a.drop_p = hp["lambda_cls"], hp["lambda_adv"], hp["p"]
        a.rng_seed = self.seed
        a.apply_adam = int(bool(apply_adam))
        a.losses = self.losses.data_ptr()
        a.logits = self.logits.data_ptr()
        a.workspace = self.workspace.data_ptr()
        a.workspace_bytes = self.workspace.numel()
        a.semi = int(bool(semi))
        a.lambda_semi, a.semi_th = hp["lambda_semi"], hp["semi_th"]
        a.part = int(part)
        a.precision = self.precision
        a.rng_rank, a.rng_world = self.rng_rank, self.rng_world
        _fill_epilogue(a, self._epilogue if part != 1 else None,
                       self._gather if part != 2 else None)
        return a

    def sync_hyper(self):
        """Re-read lr / betas / eps from the optimizers (a scheduler may have
        changed them); a graph captured before keeps the old values, so the
        trainer recaptures when they change."""
        opt, opt_d = (self.optimizers + (None,))[:2] if hasattr(self, "optimizers") else \
            (self.optimizer, None)
        if opt is not None:
            g = opt.param_groups[0]
            self.hp.update(lr=float(g["lr"]), betas=tuple(float(b) for b in g["betas"]),
                           eps=float(g["eps"]))
        if opt_d is not None:
            gd = opt_d.param_groups[0]
            if opt is not None and (tuple(float(b) for b in gd["betas"]) != self.hp["betas"]
                                    or float(gd["eps"]) != self.hp["eps"]
                                    or float(gd.get("weight_decay", 0) or 0) != 0.0):
                # the fused Adam applies ONE (betas, eps) pair to G and D (pcadv_adv_args)
                raise ValueError(
                    "the fused adversarial step applies the generator optimizer's betas / eps to "
                    "the discriminator too: optimizer_D now has betas "
                    f"{tuple(gd['betas'])}, eps {gd['eps']}, weight_decay "
                    f"{gd.get('weight_decay', 0)} against {self.hp['betas']}, {self.hp['eps']}, 0")
            self.hp["lr_D"] = float(gd["lr"])

    def set_rng_rank(self, rank, world):
        """Key the device draws by the global batch's rows (data parallelism)."""
        rank, world = int(rank), int(world)
        if world < 1 or not 0 <= rank < world:
            raise ValueError(f"rng rank {rank} of {world}")
        self.rng_rank, self.rng_world = rank, world

    # gradients that are final before the feature backward: g_grad[G_FC1_W:] and
    # all of D, contiguous in grad_flat (part 1 of a split step)
    supports_parts = True

    def early_grads(self):
        return self.grad_flat[G_LATE_END:]

    def late_grads(self):
        return self.grad_flat[:G_LATE_END]

    def __call__(self, pts_gt, labels, pts_nogt, masks=None, soft=None, apply_adam=True,
                 semi=False, part=0):
        """Whole iteration: forward, losses, backward, both Adam steps.  part=1
        stops before the feature backward, part=2 runs only the feature backward
        (and Adam when apply_adam) on the state part 1 left."""
        a = self._args(pts_gt, labels, pts_nogt, masks, soft, apply_adam, semi, part)
        check(self.lib.pcadv_adv_step(ctypes.byref(a), stream_ptr()), "pcadv_adv_step")
        return self.losses

    def grads(self, pts_gt, labels, pts_nogt, masks=None, soft=None, semi=False):
        """Forward + backward only (gradients in grad_flat; step counter advanced)."""
        return self(pts_gt, labels, pts_nogt, masks, soft, apply_adam=False, semi=semi)

    # adam(part=1) / adam(part=2): the parameters of the early / late gradient
    # bucket (Adam is elementwise: both together are adam() bitwise)
    supports_split_adam = True

    def adam(self, part=0):
        """optimizer.step(); optimizer_D.step() on the current gradients
        (part 1: g_param[G_LATE_END:] and D; part 2: g_param[:G_LATE_END])."""
        a = AdvArgs()
        a.part = int(part)
        a.g_param, a.g_grad = self.g_param.data_ptr(), self.g_grad.data_ptr()
        a.g_m, a.g_v = self.g_m.data_ptr(), self.g_v.data_ptr()
        a.d_param, a.d_grad = self.d_param.data_ptr(), self.d_grad.data_ptr()
        a.d_m, a.d_v = self.d_m.data_ptr(), self.d_v.data_ptr()
        a.step_count = self.step_count.data_ptr()
        a.lr_g, a.lr_d = self.hp["lr"], self.hp["lr_D"]
        a.beta1, a.beta2, a.eps = self.hp["betas"][0], self.hp["betas"][1], self.hp["eps"]
        check(self.lib.pcadv_adv_step_adam(ctypes.byref(a), stream_ptr()), "pcadv_adv_step_adam")

    # ------------------------------------------------------------------
    def _snapshot(self):
        return [t.clone() for t in (self.g_param, self.g_m, self.g_v, self.d_param, self.d_m,
                                    self.d_v, self.step_count)]

    def _restore(self, saved):
        for dst, src in zip((self.g_param, self.g_m, self.g_v, self.d_param, self.d_m, self.d_v,
                             self.step_count), saved):
            dst.copy_(src)

    def capture_on(self, pts_gt, labels, pts_nogt, apply_adam=True, semi=False, part=0):
        """Capture one step (or one part of it) reading the given (resident)
        input buffers into a HIP graph; state is left as it was before the
        capture."""
        saved = self._snapshot()
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up: the whole step (part 2 needs part 1's state)
            self(pts_gt, labels, pts_nogt, apply_adam=apply_adam, semi=semi)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        a = self._args(pts_gt, labels, pts_nogt, None, None, apply_adam, semi, part)
        self._keep.append(a)
        with torch.cuda.graph(g):
            check(self.lib.pcadv_adv_step(ctypes.byref(a), stream_ptr()), "pcadv_adv_step (capture)")
        torch.cuda.synchronize()
        self._restore(saved)
        return g

    def capture_seq(self, batches, apply_adam=True):
        """Capture len(batches) consecutive steps, step i reading the resident
        buffers batches[i] = (pts_gt, labels, pts_nogt), into ONE HIP graph (the
        device step counter advances per step, so each draws its own dropout
        masks and D labels).  One replay = len(batches) iterations with one
        graph-launch overhead; state is left as it was before the capture."""
        saved = self._snapshot()
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self(*batches[0], apply_adam=apply_adam)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        args = [self._args(pg, lab, pn, None, None, apply_adam, False, 0) for pg, lab, pn in batches]
        self._keep.extend(args)
        with torch.cuda.graph(g):
            for a in args:
                check(self.lib.pcadv_adv_step(ctypes.byref(a), stream_ptr()), "pcadv_adv_step (capture)")
        torch.cuda.synchronize()
        self._restore(saved)
        return g

    def capture(self):
        """Capture one step over static input buffers; returns the buffers
        (pts_gt, labels, pts_nogt) to fill before replay()."""
        B, N, dev = self.B, self.N, self.device
        st = (torch.zeros(B, N, 3, device=dev), torch.zeros(B, device=dev, dtype=torch.int64),
              torch.zeros(B, N, 3, device=dev))
        self._static = st
        self.graph = self.capture_on(*st)
        return st

    def replay(self):
        self.graph.replay()
        return self.losses

    # ------------------------------------------------------------------
    def saved_x3(self):
        """conv3 activations of the last step, (2B, N, 128) view of the workspace
        (first region of the carve in csrc/capi.hip): float32, or bfloat16 in
        bf16 mode (the form the feature backward read)."""
        C, N = 2 * self.B, self.N
        n = C * N * 128
        if self.precision == 1:
            return self.workspace[:2 * n].view(torch.bfloat16).view(C, N, 128)
        return self.workspace[:4 * n].view(torch.float32).view(C, N, 128)

    def sync_optimizer_state(self):
        """Copy the device step counter into the torch optimizers' 'step'."""
        t = float(self.step_count.item())
        for opt in self.optimizers:
            set_optimizer_step(opt, t)

    def after_torch_step(self):
        """After an iteration the trainer ran through autograd and the torch
        optimizers (unequal GT / no-GT batches): the device step counter
        advances with torch's, and each p.grad (a fresh tensor after
        zero_grad + backward) is copied back into the flat gradient buffer
        and rebound as its view."""
        self.step_count += 1
        for opt, mod, m, v, gr, layout in self._bind:
            gv = _views(gr, mod, layout)
            for name, p in mod.named_parameters():
                if p.grad is None:
                    gv[name].zero_()  # no gradient this iteration: not the last fused one's
                elif p.grad.data_ptr() != gv[name].data_ptr():
                    gv[name].copy_(p.grad)
                p.grad = gv[name]


def ft_layout(model):
    """Flat layout of a PointNetCls(feature_transform=True): the plain
    generator's tensors at their include/pcadv.h offsets (so the fused tail's
    fc1..fc3 offsets hold), then the STNkd(64) parameters in state_dict order,
    each 256-B aligned.  Returns (layout, numel)."""
    layout = dict(G_LAYOUT)
    off = (G_NUMEL + 63) // 64 * 64
    for name, p in model.named_parameters():
        if name in layout:
            continue
        layout[name] = off
        off += (p.numel() + 63) // 64 * 64
    return layout, off


def _ft_extractor_forward(P, pts, N):
    """PointNetfeat(feature_transform=True) forward (models/pointnet.py:109-130)
    on the point-wise kernels over C clouds of N points: conv1 -> conv2 ->
    STNkd(64) (conv 64 -> 64 -> 128, conv 128 -> 1024 + ReLU + max, fc1 .. fc3
    + I) -> x2 T -> conv3 -> conv4 + max.  P: the generator's parameters by
    name.  Returns every activation the backward reads."""
    from . import ops
    from .ops import ACT_NONE as NONE, ACT_RELU as RELU
    C = pts.shape[0]
    s = "feat.fstn."
    if _FT_CHAIN:  # conv1 -> conv2 -> STNkd conv1 -> conv2 in one launch
        x1, x2, h1, h2 = ops.pw_chain(pts, [
            (P["feat.conv1.weight"], P["feat.conv1.bias"], RELU, False, 0),
            (P["feat.conv2.weight"], P["feat.conv2.bias"], RELU, False, 0),
            (P[s + "conv1.weight"], P[s + "conv1.bias"], RELU, False, 0),
            (P[s + "conv2.weight"], P[s + "conv2.bias"], RELU, False, 0)])
    else:
        x1 = ops.pw_fwd(pts, P["feat.conv1.weight"], P["feat.conv1.bias"], RELU)
        x2 = ops.pw_fwd(x1, P["feat.conv2.weight"], P["feat.conv2.bias"], RELU)
        h1 = ops.pw_fwd(x2, P[s + "conv1.weight"], P[s + "conv1.bias"], RELU)
        h2 = ops.pw_fwd(h1, P[s + "conv2.weight"], P[s + "conv2.bias"], RELU)
    gs, gis = ops.conv_max_fwd(h2, P[s + "conv3.weight"], P[s + "conv3.bias"], True)
    f1 = ops.linear_fwd(gs, P[s + "fc1.weight"], P[s + "fc1.bias"], RELU)
    f2 = ops.linear_fwd(f1, P[s + "fc2.weight"], P[s + "fc2.bias"], RELU)
    t = ops.linear_fwd(f2, P[s + "fc3.weight"], P[s + "fc3.bias"], NONE, add_identity_k=64)
    T = t.view(C, 64, 64)
    if _FT_CHAIN:  # the transform x2 T and conv3 in one launch
        x2t, x3 = ops.pw_chain(x2, [(T, None, NONE, True, N),
                                    (P["feat.conv3.weight"], P["feat.conv3.bias"], RELU,
                                     False, 0)])
    else:
        x2t = ops.pw_fwd(x2, T, None, NONE, kmajor=True, rows_per_w=N)
        x3 = ops.pw_fwd(x2t, P["feat.conv3.weight"], P["feat.conv3.bias"], RELU)
    gmax, gidx = ops.conv_max_fwd(x3, P["feat.conv4.weight"], P["feat.conv4.bias"], False)
    return dict(x1=x1, x2=x2, h1=h1, h2=h2, gs=gs, gis=gis, f1=f1, f2=f2, t=t, T=T, x2t=x2t,
                x3=x3, gmax=gmax, gidx=gidx)


def _ft_extractor_backward(P, Gr, act, pts, dgmax, N, dT_hook=None):
    """The extractor's backward by hand from dL/dgmax: sparse max-pool
    backwards, dT = x2^T dx2t and dx2 = dx2t T^T per cloud (dT_hook(dT) then
    adds the regulariser's gradient in place when it joins the loss), STNkd's
    backward, its input gradient added into conv2's; weight gradients written
    into the flat gradient views Gr, the five point-wise ones' slab sums in
    one launch."""
    from . import ops
    from .ops import ACT_NONE as NONE, ACT_RELU as RELU, _mat
    C = pts.shape[0]
    s = "feat.fstn."
    x1, x2, h1, h2, gs, gis = act["x1"], act["x2"], act["h1"], act["h2"], act["gs"], act["gis"]
    f1, f2, t, T, x2t, x3, gidx = (act["f1"], act["f2"], act["t"], act["T"], act["x2t"], act["x3"],
                                   act["gidx"])
    jobs = []
    # dz3 = dx3 [x3 > 0] straight from the max-pool backward (its dx rows
    # already carry conv3's ReLU mask: conv3's backward reads no x3)
    dz3, _, _ = ops.conv_max_bwd(dgmax, gidx, x3, P["feat.conv4.weight"],
                                 dw_out=Gr["feat.conv4.weight"], db_out=Gr["feat.conv4.bias"],
                                 dx_relu=True)
    w3 = _mat(P["feat.conv3.weight"])
    dx2t = ops.pw_bwd_data(dz3, None, NONE, w3, 64)
    ops.pw_bwd_weight(dz3, None, NONE, x2t, dw_out=Gr["feat.conv3.weight"],
                      db_out=Gr["feat.conv3.bias"], defer=jobs)
    # x2t = x2 T: dT = x2^T dx2t per cloud, dx2 = dx2t T^T
    dT, _ = ops.pw_bwd_weight(dx2t, None, NONE, x2, rows_per_group=N, kmajor=True, need_db=False)
    if dT_hook is not None:
        dT_hook(dT)
    dx2 = ops.pw_bwd_data(dx2t, None, NONE, T, 64, kmajor=True, rows_per_w=N)
    # STNkd backward (models/pointnet.py:59-79); the identity add has no gradient
    df2, _, _ = ops.linear_bwd(dT.view(C, 64 * 64), t, NONE, None, 0.0, f2, P[s + "fc3.weight"],
                               dw_out=Gr[s + "fc3.weight"], db_out=Gr[s + "fc3.bias"])
    df1, _, _ = ops.linear_bwd(df2, f2, RELU, None, 0.0, f1, P[s + "fc2.weight"],
                               dw_out=Gr[s + "fc2.weight"], db_out=Gr[s + "fc2.bias"])
    dgs, _, _ = ops.linear_bwd(df1, f1, RELU, None, 0.0, gs, P[s + "fc1.weight"],
                               dw_out=Gr[s + "fc1.weight"], db_out=Gr[s + "fc1.bias"])
    dzh2, _, _ = ops.conv_max_bwd(dgs, gis, h2, P[s + "conv3.weight"], gmax_relu=gs,
                                  dw_out=Gr[s + "conv3.weight"], db_out=Gr[s + "conv3.bias"],
                                  dx_relu=True)
    dh1 = ops.pw_bwd_data(dzh2, None, NONE, _mat(P[s + "conv2.weight"]), 64)
    ops.pw_bwd_weight(dzh2, None, NONE, h1, dw_out=Gr[s + "conv2.weight"],
                      db_out=Gr[s + "conv2.bias"], defer=jobs)
    ops.pw_bwd_data(dh1, h1, RELU, _mat(P[s + "conv1.weight"]), 64, out=dx2)
    ops.pw_bwd_weight(dh1, h1, RELU, x2, dw_out=Gr[s + "conv1.weight"],
                      db_out=Gr[s + "conv1.bias"], defer=jobs)
    dx1 = ops.pw_bwd_data(dx2, x2, RELU, _mat(P["feat.conv2.weight"]), 64)
    ops.pw_bwd_weight(dx2, x2, RELU, x1, dw_out=Gr["feat.conv2.weight"],
                      db_out=Gr["feat.conv2.bias"], defer=jobs)
    ops.pw_bwd_weight(dx1, x1, RELU, pts, dw_out=Gr["feat.conv1.weight"],
                      db_out=Gr["feat.conv1.bias"], defer=jobs)
    ops.pw_wgrad_finish(jobs)


class AdvFtTrainStep(AdvTrainStep):
    """run_training's iteration (utils/trainer.py:426-559) with a
    PointNetCls(k=40, feature_transform=True) generator + DeepConvDiscNet(40, 1)
    (VERDICT r05 item 4), without autograd:

    * the generator's feature extractor over BOTH batches as one C = 2B
      pass on the point-wise kernels: conv1, conv2, STNkd(64) (conv 64->64->128,
      conv 128->1024 + ReLU + max on k_conv4_max, fc1..fc3 + I), the transform
      x2 T (models/pointnet.py:118-122), conv3, conv4 + max;
    * everything from fc1 on - head, dropout, log_softmax / CE, the three D
      passes and their BCE terms, D's gradients, the head backward - is the
      fused step's own tail (pcadv_adv_step part 3, the same launches as the
      plain step), returning dL/dgmax;
    * the backward of the extractor by hand (sparse max-pool backwards, the
      transform's dT = x2^T dx2t and dx2 = dx2t T^T, STNkd's backward, its
      input gradient added into conv2's), weight gradients written straight
      into the flat gradient buffer;
    * both Adam updates in one launch (pcadv_adam2).

    The regulariser is not part of run_training's loss (the reference leaves
    it commented out, utils/trainer.py:473-476, :511-517).  Parameters,
    gradients, Adam moments and the device draws are laid out and keyed as in
    AdvTrainStep (ft_layout for the generator), so the trainer's graphed
    iteration, checkpoints and the torch optimizers' state work unchanged."""

    supports_parts = False

    def __init__(self, model, model_D, B, N, optimizer=None, optimizer_D=None, lr=1e-4,
                 lr_D=1e-4, betas=(0.9, 0.999), eps=1e-8, lambda_cls=1.0, lambda_adv=0.001,
                 seed=0, device="cuda", lambda_semi=1.0, semi_th=0.8, rng_rank=0, rng_world=1):
        self.lib = _lib.load()
        if not getattr(model, "feature_transform", False):
            raise ValueError("AdvFtTrainStep: the generator has no feature transform "
                             "(use AdvTrainStep)")
        self.set_rng_rank(rng_rank, rng_world)
        self.model, self.model_D = model, model_D
        self.precision = 0
        self.B, self.N = int(B), int(N)
        if self.N % 128:
            # the per-cloud transform x2 T and its dT = x2^T dx2t run on 64- / 128-row
            # tiles (pcadv_pw_fwd rows_per_w, pcadv_pw_bwd_weight rows_per_group)
            raise ValueError(f"AdvFtTrainStep: N = {self.N} points, a multiple of 128 is required")
        dev = torch.device(device)
        if dev.type != "cuda":
            raise ValueError("AdvFtTrainStep runs on the HIP device only")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        if optimizer is not None:
            g = optimizer.param_groups[0]
            lr, betas, eps = g["lr"], tuple(g["betas"]), g["eps"]
        if optimizer_D is not None:
            lr_D = optimizer_D.param_groups[0]["lr"]
        self.hp = dict(lr=float(lr), lr_D=float(lr_D), betas=tuple(float(b) for b in betas),
                       eps=float(eps), lambda_cls=float(lambda_cls),
                       lambda_adv=float(lambda_adv), p=float(model.dropout.p),
                       lambda_semi=float(lambda_semi), semi_th=float(semi_th))
        self.layout, self.g_numel = ft_layout(model)
        self.g_param = flatten_params(model, self.layout, self.g_numel, dev)
        self.d_param = flatten_params(model_D, D_LAYOUT, D_NUMEL, dev)
        d_off = (self.g_numel + 63) // 64 * 64
        self.grad_flat = torch.zeros(d_off + D_NUMEL, device=dev)
        self.g_grad = self.grad_flat[:self.g_numel]
        self.d_grad = self.grad_flat[d_off:]
        self.g_m = torch.zeros_like(self.g_param)
        self.g_v = torch.zeros_like(self.g_param)
        self.d_m = torch.zeros_like(self.d_param)
        self.d_v = torch.zeros_like(self.d_param)
        t0 = max(_adopt_adam_state(optimizer, model, self.g_m, self.g_v, self.layout),
                 _adopt_adam_state(optimizer_D, model_D, self.d_m, self.d_v, D_LAYOUT))
        self.step_count = torch.full((1,), t0, device=dev, dtype=torch.int32)
        self._bind = ((optimizer, model, self.g_m, self.g_v, self.g_grad, self.layout),
                      (optimizer_D, model_D, self.d_m, self.d_v, self.d_grad, D_LAYOUT))
        for args_ in self._bind:
            _bind_adam_state(*args_, t0)
        self.optimizers = (optimizer, optimizer_D)
        self.losses = torch.zeros(6, device=dev)
        self.logits = torch.zeros(2 * self.B, 40, device=dev)
        nbytes = self.lib.pcadv_adv_step_workspace_bytes(self.B, self.N)
        self.workspace = torch.empty(nbytes, device=dev, dtype=torch.uint8)
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.graph = None
        self._keep = []
        C = 2 * self.B
        self.pts = torch.empty(C, self.N, 3, device=dev)     # [GT; no-GT] clouds
        self.dgmax = torch.empty(C, 1024, device=dev)
        self._p = dict(model.named_parameters())
        self._g = _views(self.g_grad, model, self.layout)

    # the trainer's graphed iteration folds its gathers / epilogue into the
    # step; here they are this call's first and last launches
    def _pre(self):
        if self._gather is not None:
            check(self.lib.pcadv_gather_clouds_multi(self._gather, len(self._gather),
                                                     stream_ptr()), "pcadv_gather_clouds_multi")

    def _post(self):
        if self._epilogue is None:
            return
        counters, n, ring = self._epilogue
        P = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
        if ring is None:
            check(self.lib.pcadv_iter_epilogue(P(counters), n, None, 0, None, 0, None,
                                               stream_ptr()), "pcadv_iter_epilogue")
        else:
            check(self.lib.pcadv_iter_epilogue(P(counters), n, P(self.losses), ring.nl,
                                               P(ring.ring), ring.slots, P(ring.count),
                                               stream_ptr()), "pcadv_iter_epilogue")

    def __call__(self, pts_gt, labels, pts_nogt, masks=None, soft=None, apply_adam=True,
                 semi=False, part=0):
        from . import ops
        from .ops import ACT_NONE as NONE, ACT_RELU as RELU, _mat
        if part != 0:
            raise ValueError("AdvFtTrainStep: no split parts")
        a = self._args(pts_gt, labels, pts_nogt, masks, soft, False, semi, 3)
        a.gather, a.ngather = None, 0  # gathered here, not by a fused first launch
        a.epi_counters, a.epi_ncounters, a.epi_ring = None, 0, None
        B, N = int(pts_gt.shape[0]), self.N
        C = 2 * B
        P, Gr = self._p, self._g
        self._pre()
        pts = self.pts[:C]
        # [GT; no-GT] as one input and the step number advanced, in one launch
        # (two memcpy graph nodes and a counter launch cost ~24 us)
        n = B * N * 3
        check(self.lib.pcadv_concat2(pts_gt.data_ptr(), n, pts_nogt.data_ptr(), n, pts.data_ptr(),
                                     self.step_count.data_ptr(), stream_ptr()), "pcadv_concat2")
        # ---- PointNetfeat with the feature transform (pointnet.py:109-130) ----
        act = _ft_extractor_forward(P, pts, N)
        gmax = act["gmax"]
        # ---- fc1 on: the fused step's tail (part 3) -> dL/dgmax ---------------
        dgmax = self.dgmax[:C]
        a.feat_gmax, a.feat_dgmax = gmax.data_ptr(), dgmax.data_ptr()
        self._keep_last = (a, gmax)
        check(self.lib.pcadv_adv_step(ctypes.byref(a), stream_ptr()), "pcadv_adv_step (part 3)")
        # ---- the extractor's backward -------------------------------------------
        _ft_extractor_backward(P, Gr, act, pts, dgmax, N)
        if apply_adam:
            self.adam()
        self._post()
        return self.losses

    def grads(self, pts_gt, labels, pts_nogt, masks=None, soft=None, semi=False):
        return self(pts_gt, labels, pts_nogt, masks, soft, apply_adam=False, semi=semi)

    def adam(self, part=0):
        """optimizer.step(); optimizer_D.step() (utils/trainer.py:558-559) at the
        step number this iteration's tail advanced."""
        if part != 0:
            raise ValueError("AdvFtTrainStep: no split Adam")
        hp = self.hp
        check(self.lib.pcadv_adam2(self.g_param.data_ptr(), self.g_grad.data_ptr(),
                                   self.g_m.data_ptr(), self.g_v.data_ptr(), self.g_numel,
                                   hp["lr"], self.d_param.data_ptr(), self.d_grad.data_ptr(),
                                   self.d_m.data_ptr(), self.d_v.data_ptr(), D_NUMEL, hp["lr_D"],
                                   self.step_count.data_ptr(), hp["betas"][0], hp["betas"][1],
                                   hp["eps"], stream_ptr()), "pcadv_adam2")

    def capture_on(self, pts_gt, labels, pts_nogt, apply_adam=True, semi=False, part=0):
        """One iteration over resident input buffers as a HIP graph (state left
        as it was before the capture)."""
        saved = self._snapshot()
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self(pts_gt, labels, pts_nogt, apply_adam=apply_adam, semi=semi)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self(pts_gt, labels, pts_nogt, apply_adam=apply_adam, semi=semi)
        torch.cuda.synchronize()
        self._restore(saved)
        return g

    def capture_seq(self, batches, apply_adam=True):
        raise NotImplementedError("AdvFtTrainStep: one iteration per graph")

    def saved_x3(self):
        raise NotImplementedError("AdvFtTrainStep keeps no x3 in its workspace")


class ClsTrainStep:
    """run_training_pointnet_cls's iteration (utils/trainer.py:222-268) for
    PointNetCls(k=40, feature_transform=False): forward on B labelled clouds,
    lambda_cls * CrossEntropyLoss, backward, Adam - one pcadv_cls_step call
    (BASELINE configs[1]).  Parameters, gradients and Adam moments are flat
    buffers as in AdvTrainStep; returns the device tensor [loss_cls].
    precision="bf16": the feature forward's conv3 / conv4 on bf16-rounded
    operands (configs[1] is quoted in bf16); everything else f32."""

    _epilogue = None  # (counters, ncounters, _LossRing) folded into the last launch
    _gather = None    # ctypes GatherJob array gathered by the first launch

    @contextlib.contextmanager
    def folded_epilogue(self, counters=None, ncounters=0, ring=None):
        """Within the block every step call also runs the training iteration's
        epilogue (counters[:ncounters] += 1, the losses into the loss ring; as
        pcadv_iter_epilogue) inside its own finishing launch - one launch less
        per graph-replayed iteration (pcadv_adv_args.epi_*)."""
        self._epilogue = (counters, int(ncounters), ring)
        try:
            yield
        finally:
            self._epilogue = None

    @contextlib.contextmanager
    def folded_gather(self, jobs):
        """Within the block every step call gathers its own input batches in
        its first launch (pcadv_adv_args.gather: the loaders' gather_at jobs,
        DeviceCloudLoader._gather_job, whose outputs are the step's inputs) -
        the iteration's gather launch disappears."""
        self._gather = (_lib.GatherJob * len(jobs))(*jobs)
        try:
            yield
        finally:
            self._gather = None

    def __init__(self, model, B, N, optimizer=None, lr=1e-4, betas=(0.9, 0.999), eps=1e-8,
                 lambda_cls=1.0, seed=0, device="cuda", precision="fp32", rng_rank=0, rng_world=1):
        self.lib = _lib.load()
        self.set_rng_rank(rng_rank, rng_world)
        self.model = model
        self.precision = _precision(precision)
        self.B, self.N = int(B), int(N)
        dev = torch.device(device)
        if dev.type != "cuda":
            raise ValueError("ClsTrainStep runs on the HIP device only")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        if getattr(model, "feature_transform", False):
            raise NotImplementedError("ClsTrainStep: feature_transform=True trains through "
                                      "run_training_pointnet_cls's autograd path")
        if optimizer is not None:
            g = optimizer.param_groups[0]
            lr, betas, eps = g["lr"], tuple(g["betas"]), g["eps"]
        self.hp = dict(lr=float(lr), betas=betas, eps=float(eps), lambda_cls=float(lambda_cls),
                       p=float(model.dropout.p))
        self.g_param = flatten_params(model, G_LAYOUT, G_NUMEL, dev)
        self.g_grad = torch.zeros(G_NUMEL, device=dev)
        self.g_m = torch.zeros_like(self.g_param)
        self.g_v = torch.zeros_like(self.g_param)
        t0 = _adopt_adam_state(optimizer, model, self.g_m, self.g_v, G_LAYOUT)
        self.step_count = torch.full((1,), t0, device=dev, dtype=torch.int32)
        _bind_adam_state(optimizer, model, self.g_m, self.g_v, self.g_grad, G_LAYOUT, t0)
        self._bind = ((optimizer, model, self.g_m, self.g_v, self.g_grad, G_LAYOUT),)
        self.optimizer = optimizer
        self.losses = torch.zeros(1, device=dev)
        self.logits = torch.zeros(self.B, 40, device=dev)
        nbytes = self.lib.pcadv_adv_step_workspace_bytes(self.B, self.N)
        self.workspace = torch.empty(nbytes, device=dev, dtype=torch.uint8)
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self._keep = []

    def _args(self, pts, labels, mask, apply_adam):
        B, N = int(pts.shape[0]), self.N
        if not 0 < B <= self.B:
            raise ValueError(f"batch of {B} clouds; this step was built for at most {self.B}")
        for t, nm, shape, dt in ((pts, "pts", (B, N, 3), torch.float32),
                                 (labels, "labels", (B,), torch.int64)):
            if (tuple(t.shape) != shape or t.dtype != dt or not t.is_contiguous()
                    or t.device != self.device):
                raise ValueError(f"{nm}: expected contiguous {dt} {shape} on {self.device}")
        a = AdvArgs()
        a.B, a.N = B, N
        a.pts_gt, a.labels = pts.data_ptr(), labels.data_ptr()
        if mask is not None:
            if tuple(mask.shape) != (B, 256) or mask.dtype != torch.float32 or not mask.is_contiguous():
                raise ValueError("dropout mask must be contiguous float32 (B, 256)")
            a.drop_mask_gt = mask.data_ptr()
        a.g_param, a.g_grad = self.g_param.data_ptr(), self.g_grad.data_ptr()
        a.g_m, a.g_v = self.g_m.data_ptr(), self.g_v.data_ptr()
        a.step_count = self.step_count.data_ptr()
        hp = self.hp
        a.lr_g, a.beta1, a.beta2, a.eps = hp["lr"], hp["betas"][0], hp["betas"][1], hp["eps"]
        a.lambda_cls, a.drop_p = hp["lambda_cls"], hp["p"]
        a.rng_seed = self.seed
        a.apply_adam = int(bool(apply_adam))
        a.losses = self.losses.data_ptr()
        a.logits = self.logits.data_ptr()
        a.workspace = self.workspace.data_ptr()
        a.workspace_bytes = self.workspace.numel()
        a.precision = self.precision
        a.rng_rank, a.rng_world = self.rng_rank, self.rng_world
        _fill_epilogue(a, self._epilogue, self._gather)
        return a

    set_rng_rank = AdvTrainStep.set_rng_rank
    sync_hyper = AdvTrainStep.sync_hyper

    def __call__(self, pts, labels, mask=None, apply_adam=True):
        a = self._args(pts, labels, mask, apply_adam)
        check(self.lib.pcadv_cls_step(ctypes.byref(a), stream_ptr()), "pcadv_cls_step")
        return self.losses

    def capture_on(self, pts, labels):
        """A HIP graph of one step over resident buffers (state restored)."""
        saved = [t.clone() for t in (self.g_param, self.g_m, self.g_v, self.step_count)]
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self(pts, labels)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        a = self._args(pts, labels, None, True)
        self._keep.append(a)
        with torch.cuda.graph(g):
            check(self.lib.pcadv_cls_step(ctypes.byref(a), stream_ptr()), "pcadv_cls_step (capture)")
        torch.cuda.synchronize()
        for dst, src in zip((self.g_param, self.g_m, self.g_v, self.step_count), saved):
            dst.copy_(src)
        return g

    def capture_seq(self, batches):
        """len(batches) consecutive steps (batches[i] = (pts, labels)) in ONE
        HIP graph, as AdvTrainStep.capture_seq (state restored)."""
        saved = [t.clone() for t in (self.g_param, self.g_m, self.g_v, self.step_count)]
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self(*batches[0])
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        args = [self._args(pts, lab, None, True) for pts, lab in batches]
        self._keep.extend(args)
        with torch.cuda.graph(g):
            for a in args:
                check(self.lib.pcadv_cls_step(ctypes.byref(a), stream_ptr()), "pcadv_cls_step (capture)")
        torch.cuda.synchronize()
        for dst, src in zip((self.g_param, self.g_m, self.g_v, self.step_count), saved):
            dst.copy_(src)
        return g

    def sync_optimizer_state(self):
        if self.optimizer is not None:
            set_optimizer_step(self.optimizer, float(self.step_count.item()))

    after_torch_step = AdvTrainStep.after_torch_step


class ClsFtTrainStep(ClsTrainStep):
    """run_training_pointnet_cls's iteration (utils/trainer.py:222-268) with
    PointNetCls(k=40, feature_transform=True), without autograd: the
    extractor's forward on the point-wise kernels (_ft_extractor_forward: two
    chained launches, STNkd, the transform), the cls step's head on those
    pooled features (pcadv_cls_step part 3: fc1, fc2 + dropout, fc3 + CE and
    lambda_cls dCE back to dL/dgmax), feature_transform_regularizer(T) and
    lambda_regu times its gradient (models/pointnet.py:345-353, trainer.py:
    259-266), the extractor's backward by hand, one Adam launch.  losses =
    [loss_cls, loss_regu] (the two values the reference logs).  Parameters,
    gradients and Adam moments are flat buffers in ft_layout order bound to
    the model and optimizer as ClsTrainStep's."""

    def __init__(self, model, B, N, optimizer=None, lr=1e-4, betas=(0.9, 0.999), eps=1e-8,
                 lambda_cls=1.0, lambda_regu=0.001, seed=0, device="cuda", rng_rank=0,
                 rng_world=1):
        self.lib = _lib.load()
        self.set_rng_rank(rng_rank, rng_world)
        if not getattr(model, "feature_transform", False):
            raise ValueError("ClsFtTrainStep: the model has no feature transform (use ClsTrainStep)")
        self.model = model
        self.precision = 0
        self.B, self.N = int(B), int(N)
        if self.N % 128:
            raise ValueError(f"ClsFtTrainStep: N = {self.N} points, a multiple of 128 is required")
        dev = torch.device(device)
        if dev.type != "cuda":
            raise ValueError("ClsFtTrainStep runs on the HIP device only")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        if optimizer is not None:
            g = optimizer.param_groups[0]
            lr, betas, eps = g["lr"], tuple(g["betas"]), g["eps"]
        self.hp = dict(lr=float(lr), betas=tuple(float(b) for b in betas), eps=float(eps),
                       lambda_cls=float(lambda_cls), p=float(model.dropout.p))
        self.layout, self.g_numel = ft_layout(model)
        self.g_param = flatten_params(model, self.layout, self.g_numel, dev)
        self.g_grad = torch.zeros(self.g_numel, device=dev)
        self.g_m = torch.zeros_like(self.g_param)
        self.g_v = torch.zeros_like(self.g_param)
        t0 = _adopt_adam_state(optimizer, model, self.g_m, self.g_v, self.layout)
        self.step_count = torch.full((1,), t0, device=dev, dtype=torch.int32)
        _bind_adam_state(optimizer, model, self.g_m, self.g_v, self.g_grad, self.layout, t0)
        self._bind = ((optimizer, model, self.g_m, self.g_v, self.g_grad, self.layout),)
        self.optimizer = optimizer
        self.losses = torch.zeros(2, device=dev)  # [loss_cls, loss_regu]
        self.logits = torch.zeros(self.B, 40, device=dev)
        nbytes = self.lib.pcadv_adv_step_workspace_bytes(self.B, self.N)
        self.workspace = torch.empty(nbytes, device=dev, dtype=torch.uint8)
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self._keep = []
        self.dgmax = torch.empty(self.B, 1024, device=dev)
        self._norms = torch.empty(self.B, device=dev)
        self._lregu = torch.full((1,), float(lambda_regu), device=dev)
        self._p = dict(model.named_parameters())
        self._g = _views(self.g_grad, model, self.layout)

    @property
    def lambda_regu(self):
        return float(self._lregu.item())

    # gathers / epilogue as this call's own first and last launches
    _pre = AdvFtTrainStep._pre
    _post = AdvFtTrainStep._post

    def __call__(self, pts, labels, mask=None, apply_adam=True):
        a = self._args(pts, labels, mask, False)
        a.part = 3
        a.gather, a.ngather = None, 0
        a.epi_counters, a.epi_ncounters, a.epi_ring = None, 0, None
        B, N = int(pts.shape[0]), self.N
        P, Gr = self._p, self._g
        self._pre()
        act = _ft_extractor_forward(P, pts, N)
        # fc1 .. CE and back to dL/dgmax: the cls step's head (part 3); its
        # dropout draws read the step count of the completed steps
        dgmax = self.dgmax[:B]
        a.feat_gmax, a.feat_dgmax = act["gmax"].data_ptr(), dgmax.data_ptr()
        self._keep_last = (a, act["gmax"])
        check(self.lib.pcadv_cls_step(ctypes.byref(a), stream_ptr()), "pcadv_cls_step (part 3)")
        # loss += lambda_regu * ||T T^T - I||_F mean (trainer.py:259-266): its
        # value into losses[1], lambda_regu times its gradient added into the
        # bmm's dT, and (with Adam) the step count advanced, in one launch + the mean
        T = act["T"]

        def regulariser(dT):
            check(self.lib.pcadv_tnet_reg_step(
                T.data_ptr(), B, 64, self._norms.data_ptr(), self.losses.data_ptr() + 4,
                self._lregu.data_ptr(), dT.data_ptr(),
                self.step_count.data_ptr() if apply_adam else None, stream_ptr()),
                "pcadv_tnet_reg_step")
        _ft_extractor_backward(P, Gr, act, pts, dgmax, N, dT_hook=regulariser)
        if apply_adam:  # optimizer.step() at the count advanced above
            hp = self.hp
            check(self.lib.pcadv_adam2(self.g_param.data_ptr(), self.g_grad.data_ptr(),
                                       self.g_m.data_ptr(), self.g_v.data_ptr(), self.g_numel,
                                       hp["lr"], None, None, None, None, 0, 0.0,
                                       self.step_count.data_ptr(), hp["betas"][0],
                                       hp["betas"][1], hp["eps"], stream_ptr()), "pcadv_adam2")
        self._post()
        return self.losses

    def capture_on(self, pts, labels):
        """One iteration over resident buffers as a HIP graph (state restored)."""
        saved = [t.clone() for t in (self.g_param, self.g_m, self.g_v, self.step_count)]
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self(pts, labels)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self(pts, labels)
        torch.cuda.synchronize()
        for dst, src in zip((self.g_param, self.g_m, self.g_v, self.step_count), saved):
            dst.copy_(src)
        return g

    def capture_seq(self, batches):
        raise NotImplementedError("ClsFtTrainStep: one iteration per graph")
