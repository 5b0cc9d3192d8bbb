#!/usr/bin/env python3
"""Throughput of the adversarial train step (utils/trainer.py:run_training, one
iteration = :426-559) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-graph] [--no-cpu]

Workload (BASELINE.json configs[2]): PointNetCls(k=40) + DeepConvDiscNet(40,1),
B=32 labelled + B=32 unlabelled ModelNet40-shaped clouds of N=1024 points per
GPU per step, fp32, Adam on both networks.  Synthetic seeded inputs
(U(-1,1) points, labels in [0,40)), resident in HBM before timing starts.
metric value = whole-job clouds/s counting 2B clouds per step per rank.
--gpus N > 1: one process per GPU, each rank takes its own shard of the global
batch and gradients are averaged with an RCCL all-reduce (see DESIGN.md,
multi-GPU).  Under torch.distributed.run the ranks come from the environment
(WORLD_SIZE must equal --gpus); run directly, bench.py spawns the N ranks
itself before anything touches the GPU.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

# This entry point opts in to graph replay through the stream dispatch path
# (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0, the same as the package's
# use_stream_graph_dispatch(); importing the package never sets it).  It must
# be in the environment before torch initialises HIP; the JSON line records it
# ("runtime").  --runtime-graph-dispatch keeps the HIP runtime's default.
if "--runtime-graph-dispatch" not in sys.argv:
    os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
import torch  # noqa: E402

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

B, N = 32, 1024
POOL = 4

def _with_runtime(line):
    """The HIP runtime setting the graphs were replayed under."""
    line["runtime"] = {"DEBUG_CLR_GRAPH_PACKET_CAPTURE":
                       os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "runtime default")}
    return line
  # distinct resident input batches cycled by the timed loop


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--graph-steps", type=int, default=1,
                    help="steps captured per HIP graph (adv / cls, one GPU): a replay runs that "
                         "many consecutive iterations over the resident batch pool; a timed "
                         "region still runs exactly --steps steps (the remainder as one-step "
                         "graphs)")
    ap.add_argument("--repeats", type=int, default=3,
                    help="timed regions of --steps steps each; the median is reported")
    ap.add_argument("--points", type=int, default=1024,
                    help="points per cloud of the adv step (1024: the metric's config; 2048: "
                         "BASELINE configs[4]'s per-rank shape)")
    ap.add_argument("--config", choices=["adv", "seg", "cls", "cls_ft", "adv_ft", "trainer", "dp1"], default="adv",
                    help="adv: the headline adversarial cls step (default); seg: the "
                         "PointNetSeg training step of BASELINE configs[3]; cls: the "
                         "supervised PointNetCls step of configs[1]; cls_ft: the same with "
                         "feature_transform=True (STNkd(64) + regulariser, layer-by-layer "
                         "kernels through autograd); adv_ft: the adversarial iteration with "
                         "that generator (autograd body, graphed); trainer: run_training end to end over "
                         "DeviceCloudLoaders; dp1: the data-parallel iteration's overhead on a one-rank "
                         "RCCL group against the plain step graph")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default=None,
                    help="feature-forward precision (default: bf16 for --config cls, the dtype "
                         "BASELINE configs[1] names; fp32 for adv and seg)")
    ap.add_argument("--ft-body", action="store_true",
                    help="--config adv_ft: time the autograd body (trainer._AutogradAdvStep, "
                         "run_training with args.fused_ft = False) instead of the fused "
                         "feature-transform step")
    ap.add_argument("--runtime-graph-dispatch", action="store_true",
                    help="leave DEBUG_CLR_GRAPH_PACKET_CAPTURE unset (the HIP runtime's default "
                         "graph dispatch) instead of the stream dispatch path this bench opts in to")
    ap.add_argument("--launch-check", action="store_true",
                    help="launcher self-test: start the --gpus ranks, form the process group, "
                         "print the JSON world/backend line; no GPU work")
    return ap.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_entry(local_rank, world, port, argv):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.argv = argv
    main()


def spawn_ranks(world):
    """bench.py --gpus N run without a launcher: start N rank processes (fresh
    interpreters, spawn start method) with the torch.distributed.run
    environment.  Called before this process makes any GPU call."""
    import torch.multiprocessing as mp
    mp.spawn(_rank_entry, args=(world, _free_port(), list(sys.argv)), nprocs=world, join=True)


def _backend():
    # RCCL; PCADV_BENCH_BACKEND=gloo rehearses the multi-rank path with several
    # ranks on one GPU (RCCL needs a device per rank) - never for measurements
    return os.environ.get("PCADV_BENCH_BACKEND", "nccl")


def launch_check(args, world, rank):
    """The launcher's self-test: the process group forms with --gpus ranks."""
    import torch.distributed as tdist
    if world > 1:
        tdist.init_process_group("gloo")
        t = torch.ones(1)
        tdist.all_reduce(t)
        assert int(t.item()) == world
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "world_size": world,
                          "check_backend": "gloo" if world > 1 else None,
                          "bench_backend": _backend() if world > 1 else None,
                          "launcher": "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ
                          else ("bench.py spawn" if world > 1 else "single process")}), flush=True)
    if world > 1:
        tdist.destroy_process_group()


def make_models(dev, seed=0):
    import adversarial_learning_on_pointclouds_amd as pc
    torch.manual_seed(seed)
    model = pc.PointNetCls(k=40).to(dev)
    model_D = pc.DeepConvDiscNet(40, 1).to(dev)
    from adversarial_learning_on_pointclouds_amd.model_utils import init_weights
    init_weights(model_D, "xavier", verbose=False)
    return model, model_D


def _time_adv_oracle(seconds, dense):
    """Steps of the numpy oracle's adversarial step (B=32+32, N) for `seconds`."""
    from oracle import pointnet_np as onp
    G = onp.make_params(onp.cls_spec(40), seed=3)
    D = onp.make_params(onp.disc_spec(40, 1), seed=4, init="xavier")
    oG, oD = onp.Adam(G), onp.Adam(D)
    rng = np.random.default_rng(1000)
    pg = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    pn = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    lab = rng.integers(0, 40, B)
    m1 = (rng.random((B, 256)) >= 0.3).astype(np.float32)
    m2 = (rng.random((B, 256)) >= 0.3).astype(np.float32)
    y1 = rng.uniform(0.7, 1.05, (B, 1)).astype(np.float32)
    y2 = rng.uniform(0.0, 0.305, (B, 1)).astype(np.float32)

    def one():
        onp.adv_step(G, D, oG, oD, pg, lab, pn, m1, m2, y1, y2, dense_max_bwd=dense)

    one()  # warm-up
    t0 = time.perf_counter()
    steps = 0
    while True:
        one()
        steps += 1
        if time.perf_counter() - t0 >= seconds and steps >= 2:
            break
    return steps, time.perf_counter() - t0


def cpu_baseline(seconds):
    """The reference's algorithm on the host cores: the numpy oracle's
    adversarial step with the conv4 + max backward in the reference autograd's
    dense form (MaxBackward zero-fill + scatter, dense Conv1d dX / dW GEMMs over
    all points: oracle.conv_max_bwd_dense), on a bounded sample of the same
    workload (B=32+32, N).  The sparse-backward port (what the GPU path
    computes) is timed beside it on a shorter sample as a secondary figure."""
    steps, dt = _time_adv_oracle(seconds, dense=True)
    s_steps, s_dt = _time_adv_oracle(max(2.0, seconds / 3), dense=False)
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    out = {"value": round(2 * B * steps / dt, 2), "unit": "clouds/s", "cores": cores,
           "kind": "port",
           "algorithm": "reference (dense MaxBackward + dense conv4 backward, as autograd runs "
                        "models/pointnet.py:128-129)",
           "sample": f"{steps} numpy-oracle adversarial steps (B=32+32, N={N}, fp32, dense max-pool "
                     f"backward) in {dt:.1f}s",
           "sparse_port_value": round(2 * B * s_steps / s_dt, 2),
           "sparse_port_sample": f"{s_steps} steps with the sparse max-pool backward in {s_dt:.1f}s"}
    # the dense port against the reference's own run_training on the same cores,
    # measured in the build container (the reference never travels to this box):
    # tools/time_reference_cpu.py -> profiles/rNN_cpu_calibration.json
    cal = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_cpu_calibration.json")))
    if cal and N == 1024:
        c = json.load(open(cal[-1]))
        if "dense_port_over_reference" in c:
            out["calibration"] = {"port_over_reference": c["dense_port_over_reference"],
                                  "sparse_port_over_reference": c["port_over_reference"],
                                  "cores": c["cores"],
                                  "reference_clouds_per_s": c["reference_run_training_clouds_per_s"],
                                  "source": os.path.relpath(cal[-1], REPO)}
    return out


def cpu_baseline_seg(seconds, Bs, Ns):
    """The numpy oracle's PointNetSeg training step (forward, per-point CE,
    backward, Adam) on a bounded sample of the seg workload: B=2 clouds of
    N=2048 points per step, timed on this host's cores."""
    from oracle import pointnet_np as onp
    P = onp.make_params(onp.seg_spec(50), seed=8, init="xavier")
    opt = onp.Adam(P)
    rng = np.random.default_rng(2000)
    b = 2
    pts = rng.uniform(-1, 1, (b, Ns, 3)).astype(np.float32)
    cls = np.zeros((b, 1, 16), np.float32)
    cls[np.arange(b), 0, rng.integers(0, 16, b)] = 1
    seg = rng.integers(0, 50, (b, Ns))

    def one():
        _, grads, _, _, _ = onp.seg_step(P, pts, cls, seg)
        opt.step(grads)

    one()  # warm-up
    t0 = time.perf_counter()
    steps = 0
    while True:
        one()
        steps += 1
        if time.perf_counter() - t0 >= seconds and steps >= 2:
            break
    dt = time.perf_counter() - t0
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    return {"value": round(b * steps / dt, 2), "unit": "clouds/s", "cores": cores, "kind": "port",
            "sample": f"{steps} numpy-oracle seg steps (B={b}, N={Ns}, fp32, forward+CE+backward+Adam) "
                      f"in {dt:.1f}s"}


def cpu_baseline_cls(seconds):
    """The numpy oracle's run_training_pointnet_cls iteration (B=32, N=1024:
    forward with a dropout mask, CE, backward, Adam) timed on the host cores."""
    from oracle import pointnet_np as onp
    G = onp.make_params(onp.cls_spec(40), seed=3)
    opt = onp.Adam(G)
    rng = np.random.default_rng(3000)
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    lab = rng.integers(0, 40, B)
    m = (rng.random((B, 256)) >= 0.3).astype(np.float32)

    def one():
        logits, _, cache = onp.cls_forward(G, pts, m)
        _, dlog = onp.cross_entropy(logits, lab)
        opt.step(onp.cls_backward(G, cache, dlog))

    one()
    t0 = time.perf_counter()
    steps = 0
    while True:
        one()
        steps += 1
        if time.perf_counter() - t0 >= seconds and steps >= 2:
            break
    dt = time.perf_counter() - t0
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    return {"value": round(B * steps / dt, 2), "unit": "clouds/s", "cores": cores, "kind": "port",
            "sample": f"{steps} numpy-oracle cls steps (B=32, N=1024, fp32) in {dt:.1f}s"}


def _time_loop(one, seconds):
    one()
    t0 = time.perf_counter()
    steps = 0
    while True:
        one()
        steps += 1
        if time.perf_counter() - t0 >= seconds and steps >= 2:
            break
    return steps, time.perf_counter() - t0


def cpu_baseline_ft(seconds, adversarial):
    """The numpy oracle's feature-transform iterations on the host cores (B=32,
    N=1024): run_training_pointnet_cls's (oracle.cls_ft_step: forward with the
    STNkd(64) transform, CE + 0.001 x regulariser, backward; Adam), or for the
    adversarial iteration two such generator passes (the GT and no-GT batches,
    as the reference runs model() twice) plus the discriminator's three
    forward and two backward passes and both Adams."""
    from oracle import pointnet_np as onp
    G = onp.make_params(onp.cls_ft_spec(40), seed=3)
    Dp = onp.make_params(onp.disc_spec(40, 1), seed=4, init="xavier")
    optG, optD = onp.Adam(G), onp.Adam(Dp)
    rng = np.random.default_rng(3000)
    pts = [rng.uniform(-1, 1, (B, N, 3)).astype(np.float32) for _ in range(2)]
    lab = rng.integers(0, 40, B)
    m = (rng.random((B, 256)) >= 0.3).astype(np.float32)

    def one():
        _, _, g, aux = onp.cls_ft_step(G, pts[0], lab, m)
        if adversarial:
            _, _, g2, aux2 = onp.cls_ft_step(G, pts[1], lab, m)
            for k in g:
                g[k] = g[k] + g2[k]
            y = np.full((B, 1), 0.9, np.float32)
            gD = None
            for logits in (aux2["logits"], aux["logits"], aux2["logits"]):
                d, acts = onp.disc_forward(Dp, onp.log_softmax(logits))
                _, dd = onp.bce_with_logits(d, y)
                gd, _ = onp.disc_backward(Dp, acts, dd)
                gD = gd if gD is None else {k: gD[k] + gd[k] for k in gD}
            optD.step(gD)
        optG.step(g)
    steps, dt = _time_loop(one, seconds)
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    clouds = (2 if adversarial else 1) * B
    what = ("adversarial feature-transform iterations (2 x cls_ft_step + 3 D passes, B=32+32)"
            if adversarial else "cls_ft_step iterations (B=32)")
    return {"value": round(clouds * steps / dt, 2), "unit": "clouds/s", "cores": cores,
            "kind": "port", "sample": f"{steps} numpy-oracle {what}, N=1024, fp32, in {dt:.1f}s"}


def ft_roofline(C):
    """The feature-transform steps' dominant kernel: the 1024-channel conv +
    max over points (k_conv4_max, twice per generator pass: STNkd conv3 and
    PointNetfeat conv4) on C clouds, timed from a graph of 50 launches on
    post-ReLU inputs; achieved = algorithmic f32 FLOPs / launch time against
    the dense bf16 MFMA peak (the pipe its split products run on)."""
    from adversarial_learning_on_pointclouds_amd import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(9)
    x = torch.relu(torch.randn(C, N, 128, device=dev, generator=g))
    w = torch.randn(1024, 128, device=dev, generator=g) * (1.0 / 128 ** 0.5)
    b = torch.zeros(1024, device=dev)
    gmax = torch.empty(C, 1024, device=dev)
    gidx = torch.empty(C, 1024, device=dev, dtype=torch.int32)
    t = _graph_time(lambda: ops.conv4_max(x, w, b, precision="fp32", out=(gmax, gidx)))
    f = 2.0 * C * N * 128 * 1024
    return {"bound": "mfma",
            "kernel": f"k_conv4_max<3> (1024-channel conv + max over points, {C} clouds x {N} "
                      "points; STNkd conv3 / PointNetfeat conv4)",
            "achieved": round(f / t / 1e12, 2), "peak": BF16_PEAK, "unit": "TFLOP/s",
            "frac": round(f / t / 1e12 / BF16_PEAK, 4),
            "issued_frac": round(3 * f / t / 1e12 / BF16_PEAK, 4),
            "traffic": None, "avg_launch_us": round(t * 1e6, 2),
            "algorithmic_flops_per_launch": f,
            "algorithmic_bytes_per_launch": C * N * 128 * 4 + 1024 * 128 * 4 + C * 1024 * 8,
            "peak_basis": "dense bf16 MFMA 2500 TF; achieved = algorithmic f32 FLOPs / HIP-event "
                          "launch time (graph of 50)"}


BF16_PEAK, F32_PEAK = 2500.0, 157.3  # dense TFLOP/s (MI355X_MICROARCH.md)


def _pmc_traffic(pattern, prefixes, only_if=True):
    """Bytes per launch (L2 -> memory, PMC FETCH_SIZE x 2 + WRITE_SIZE) of the
    named kernels, summed, from the newest committed summary matching
    profiles/<pattern> (tools/pmc_traffic.py), or (None, None)."""
    if not only_if:
        return None, None
    prof = sorted(p for p in glob.glob(os.path.join(REPO, "profiles", pattern))
                  if pattern != "r*_pmc_traffic.json"
                  or not any(t in os.path.basename(p) for t in ("_seg_", "_cls_", "_adv_ft_")))
    if not prof:
        return None, None
    kern = json.load(open(prof[-1]))["kernels"]
    names = [next((k for k in kern if k.startswith(p)), None) for p in prefixes]
    if not all(names):
        return None, None
    return round(sum(kern[n]["traffic_bytes"] for n in names)), os.path.relpath(prof[-1], REPO)


def _pmc_mfma(cfg, prefix):
    """Matrix-pipe utilisation of the named kernel from the newest committed
    profiles/r*_<cfg>_mfma.json (tools/pmc_mfma.py: SQ_VALU_MFMA_BUSY_CYCLES /
    (1024 SIMDs x GRBM_GUI_ACTIVE / 8), median over the profiled launches), or
    (None, None)."""
    prof = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_{cfg}_mfma.json")))
    if not prof:
        return None, None
    kern = json.load(open(prof[-1]))["kernels"]
    hits = [v for k, v in kern.items() if k.startswith(prefix)]
    if not hits:
        return None, None
    best = max(hits, key=lambda v: v["SQ_VALU_MFMA_BUSY_CYCLES"])
    return best["mfma_busy"], os.path.relpath(prof[-1], REPO)


def _graph_time(fn, reps=50):
    """Average device time of fn() over `reps` back-to-back calls captured in
    one HIP graph (as the kernels run inside the step graph), timed with HIP
    events on the stream the graph is launched on (the current stream)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()  # warm
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    g.replay()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / 1e3 / reps


def feat_roofline(pts_all, fw, prec, traffic_pattern=None, mfma_cfg=None):
    """The roofline block for the dominant kernel, k_conv4_max (conv4 + max over
    points, models/pointnet.py:128-130), and the same figures for the feature
    forward pair (k_point_mlp + k_conv4_max, conv1..conv4).  achieved = the
    ALGORITHMIC f32 FLOPs of the launch (2 C N 128 1024 for conv4) over its
    measured time, against the dense bf16 MFMA peak: the pipe these kernels
    run on (fp32 mode emulates each f32 product with three bf16 split products
    plus an exact f32 re-evaluation of every winner; bf16 mode one product).
    issued_frac counts the MFMA work actually issued (split products)."""
    from adversarial_learning_on_pointclouds_amd import ops
    C, Np = int(pts_all.shape[0]), int(pts_all.shape[1])
    gmax, gidx, x3 = ops.feat_fwd(pts_all, *fw, precision=prec)
    pair_s = _graph_time(lambda: ops.feat_fwd(pts_all, *fw, precision=prec))
    k2_s = _graph_time(lambda: ops.conv4_max(x3, fw[6], fw[7], precision=prec, out=(gmax, gidx)))
    f4 = 2.0 * C * Np * 128 * 1024
    f12 = 2.0 * C * Np * (3 * 64 + 64 * 64)
    f3 = 2.0 * C * Np * 64 * 128
    np3, np4 = (6, 3) if prec == "fp32" else (1, 1)  # bf16 products per f32 product
    issued4 = np4 * f4
    issued_pair = f12 * (BF16_PEAK / F32_PEAK) + np3 * f3 + np4 * f4
    xe = 4 if prec == "fp32" else 2  # bytes per x3 element (bf16 mode stores it in bf16)
    alg_bytes4 = C * Np * 128 * xe + 1024 * 128 * 4 + C * 1024 * 8
    alg_bytes_pair = C * Np * 3 * 4 + 2 * C * Np * 128 * xe + C * 1024 * 8
    traffic4, src = _pmc_traffic(traffic_pattern or "none", (f"pcadv::k_conv4_max<{np4}",),
                                 traffic_pattern is not None)
    traffic_pair, _ = _pmc_traffic(traffic_pattern or "none",
                                   (f"pcadv::k_point_mlp<{np3}", f"pcadv::k_conv4_max<{np4}"),
                                   traffic_pattern is not None)
    ach4 = f4 / k2_s / 1e12
    ach_pair = (f12 + f3 + f4) / pair_s / 1e12
    busy, busy_src = _pmc_mfma(mfma_cfg, f"k_conv4_max<{np4},") if mfma_cfg else (None, None)
    return {
        "bound": "mfma",
        "kernel": f"k_conv4_max<{np4}> (conv4 128->1024 + max over points, {C} clouds x {Np} points)",
        "achieved": round(ach4, 2), "peak": BF16_PEAK, "unit": "TFLOP/s",
        "frac": round(ach4 / BF16_PEAK, 4),
        "issued_frac": round(issued4 / k2_s / 1e12 / BF16_PEAK, 4),
        "traffic": traffic4,
        "traffic_unit": "bytes/launch (L2->memory, PMC FETCH_SIZEx2+WRITE_SIZE)",
        "traffic_source": src,
        "mfma_busy": busy,
        "mfma_busy_unit": "fraction of SIMD-cycles the matrix pipe is busy (PMC "
                          "SQ_VALU_MFMA_BUSY_CYCLES / (1024 x GRBM_GUI_ACTIVE / 8))",
        "mfma_busy_source": busy_src,
        "avg_launch_us": round(k2_s * 1e6, 2),
        "algorithmic_flops_per_launch": f4,
        "algorithmic_bytes_per_launch": alg_bytes4,
        "issued_bf16_flops_per_launch": issued4,
        "peak_basis": "dense bf16 MFMA 2500 TF (MI355X_MICROARCH.md), the pipe the kernel runs on; "
                      "achieved = algorithmic f32 FLOPs / HIP-event launch time (graph of 50)",
        "pair": {"kernel": f"k_point_mlp<{np3}> + k_conv4_max<{np4}> (conv1..conv4 + max)",
                 "avg_us": round(pair_s * 1e6, 2), "achieved": round(ach_pair, 2),
                 "frac": round(ach_pair / BF16_PEAK, 4),
                 "issued_frac": round(issued_pair / pair_s / 1e12 / BF16_PEAK, 4),
                 "algorithmic_flops": f12 + f3 + f4, "issued_bf16_equiv_flops": issued_pair,
                 "algorithmic_bytes": alg_bytes_pair, "traffic": traffic_pair,
                 "issued_note": "conv1-2's f32 FLOPs weighted 2500/157.3 (the f32 pipe's rate)"},
    }


def graph_runner(single, seq, G):
    """Per-step callable for warm-up / timed_regions over `total` steps: step
    k replays single[k % POOL] or, inside a whole group of G steps, the G-step
    graph `seq` (batches 0..G-1 of the pool) once at the group's last step."""
    def run(k, total):
        full = (total // G) * G if seq is not None else 0
        if k < full:
            if k % G == G - 1:
                seq.replay()
        else:
            single[k % POOL].replay()
    return run


def timed_regions(one, steps, repeats, dist=None):
    """`repeats` timed regions of exactly `steps` steps, each bracketed by a
    barrier + synchronize on both sides; returns the per-region seconds (max
    over ranks)."""
    out = []
    for _ in range(repeats):
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            one(k)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([dt], device=torch.cuda.current_device(), dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        out.append(dt)
    return out


def bench_cls(args):
    """BASELINE.json configs[1]: PointNetCls ModelNet40 B=32, N=1024, no
    discriminator - one run_training_pointnet_cls iteration per step
    (pcadv_cls_step), HIP-graph replayed over resident batches."""
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd.step import ClsTrainStep
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = pc.PointNetCls(k=40).to(dev)
    prec = args.precision or "bf16"
    step = ClsTrainStep(model, B, N, seed=7, device=dev, precision=prec)
    pool = []
    for k in range(POOL):
        rng = np.random.default_rng(3000 + k)
        pool.append((torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev),
                     torch.from_numpy(rng.integers(0, 40, B)).to(dev)))
    graphs = [step.capture_on(*b) for b in pool]
    G = max(1, min(args.graph_steps, POOL))
    run = graph_runner(graphs, step.capture_seq(pool[:G]) if G > 1 else None, G)
    for k in range(args.warmup):
        run(k, args.warmup)
    regions = timed_regions(lambda k: run(k, args.steps), args.steps, args.repeats)
    dt = float(np.median(regions))
    gflop = 11.18  # algorithmic FLOPs of one cfg-2 step
    loss = float(step.losses[0].item())
    fw = [model.feat.conv1.weight, model.feat.conv1.bias, model.feat.conv2.weight,
          model.feat.conv2.bias, model.feat.conv3.weight, model.feat.conv3.bias,
          model.feat.conv4.weight, model.feat.conv4.bias]
    roof = feat_roofline(pool[(args.steps - 1) % POOL][0], fw, prec,
                         "r*_cls_pmc_traffic.json" if prec == "bf16" else None,
                         "cls" if prec == "bf16" else None)
    out = {
        "metric": "point-clouds/sec (cls train step, no discriminator), B=32 N=1024 ModelNet40, 1 GPU",
        "value": round(B * args.steps / dt, 1), "unit": "clouds/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": ("bf16 (conv3 / conv4 MFMAs on bf16-rounded operands, f32 accumulate; conv1-2, "
                  "head, losses, backward and Adam f32)" if prec == "bf16" else
                  "fp32 (f32-level: conv3 / conv4 as bf16 split-product MFMAs, exact-f32 max "
                  "winners)"),
        "data": "synthetic (seeded U(-1,1) clouds, labels in [0,40); resident in HBM)",
        "config": {"workload": "run_training_pointnet_cls: PointNetCls(k=40), CE, Adam, B=32, "
                               "N=1024 (BASELINE configs[1])", "global_batch": B, "points": N,
                   "parallelism": "dp1", "hip_graph": True, "steps_per_graph": G, "precision": prec},
        "timing": {"regions_s": [round(r, 6) for r in regions], "reported": "median"},
        "roofline": roof,
        "step_flops": {"gflop_per_step": gflop,
                       "achieved_tflops": round(gflop * args.steps / dt / 1e3, 2)},
        "loss_last_step": round(loss, 5), "finite": bool(np.isfinite(loss)),
    }
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_cls(args.cpu_seconds)
    print(json.dumps(_with_runtime(out)), flush=True)


def bench_cls_ft(args):
    """run_training_pointnet_cls with PointNetCls(k=40, feature_transform=True)
    (utils/trainer.py:254-268: CE + 0.001 x the regulariser, Adam).  Default:
    the fused feature-transform cls step run_training_pointnet_cls uses
    (step.ClsFtTrainStep: the extractor's forward in chained point-wise
    launches, the cls step's head on its pooled features, the regulariser and
    the extractor backward by hand, one Adam launch), one HIP graph per
    resident batch.  --ft-body: the reference's body through autograd over the
    same kernels with torch's Adam (fused where available, else capturable),
    the path before round 6."""
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd.pointnet import feature_transform_regularizer
    from adversarial_learning_on_pointclouds_amd.step import ClsFtTrainStep
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = pc.PointNetCls(k=40, feature_transform=True).to(dev).train()
    pool = []
    for k in range(POOL):
        rng = np.random.default_rng(3000 + k)
        pool.append((torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev),
                     torch.from_numpy(rng.integers(0, 40, B)).to(dev)))
    graphs, why = [], None
    if not args.ft_body:
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, betas=(0.9, 0.999))
        adam = "fused (pcadv_adam2 over the flat generator buffer)"
        step = ClsFtTrainStep(model, B, N, optimizer=opt, lambda_regu=0.001, seed=1234, device=dev)
        if not args.no_graph:
            graphs = [step.capture_on(*p) for p in pool]
        workload = ("run_training_pointnet_cls with PointNetCls(k=40, feature_transform=True): "
                    "CE + 0.001 regulariser, Adam; fused feature-transform cls step (ClsFtTrainStep)")

        def loss_now(k):
            return float(step.losses[0].item()) + 0.001 * float(step.losses[1].item())

        def run(k):
            step(*pool[k % POOL])
    else:
        try:  # one fused multi-tensor kernel per step where this torch build has it
            opt = torch.optim.Adam(model.parameters(), lr=1e-3, betas=(0.9, 0.999), fused=True,
                                   capturable=True)
            adam = "torch.optim.Adam(fused=True, capturable=True)"
        except (RuntimeError, ValueError):
            opt = torch.optim.Adam(model.parameters(), lr=1e-3, betas=(0.9, 0.999), capturable=True)
            adam = "torch.optim.Adam(capturable=True)"
        losses = torch.zeros(POOL, device=dev)

        def body(pts, lab, k):
            opt.zero_grad()  # captured: backward's gradients become p.grad, no accumulate adds
            logits, _, trans = model(pts)
            loss = (torch.nn.functional.cross_entropy(logits, lab)
                    + 0.001 * feature_transform_regularizer(trans))
            loss.backward()
            opt.step()
            losses[k].copy_(loss.detach())

        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # autograd / optimizer state created outside any capture
            for k in range(3):
                body(*pool[k % POOL], k % POOL)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if not args.no_graph:
            try:
                kept = []  # each graph's gradient buffers (the next capture drops p.grad)
                for k in range(POOL):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        body(*pool[k], k)
                    graphs.append(g)
                    kept.append([p.grad for p in model.parameters()])
            except Exception as e:  # noqa: BLE001 - reported in the line, eager timing instead
                graphs, why = [], f"{type(e).__name__}: {e}"[:200]
                torch.cuda.synchronize()
        workload = ("run_training_pointnet_cls with PointNetCls(k=40, feature_transform=True): "
                    "CE + 0.001 regulariser, Adam, autograd over the pcadv ops")

        def loss_now(k):
            return float(losses[k % POOL].item())

        def run(k):
            body(*pool[k % POOL], k % POOL)

    def one(k):
        if graphs:
            graphs[k % POOL].replay()
        else:
            run(k)
    for k in range(args.warmup):
        one(k)
    regions = timed_regions(one, args.steps, args.repeats)
    dt = float(np.median(regions))
    loss = loss_now(args.steps - 1)
    out = {
        "metric": "point-clouds/sec (cls train step with feature_transform=True), B=32 N=1024 "
                  "ModelNet40, 1 GPU",
        "value": round(B * args.steps / dt, 1), "unit": "clouds/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "fp32 (exact-f32 MFMA point-wise layers, split-product 1024-channel conv + max "
                 "with the exact max re-evaluated, head f32)",
        "data": "synthetic (seeded U(-1,1) clouds, labels in [0,40); resident in HBM)",
        "config": {"workload": workload, "global_batch": B, "points": N,
                   "parallelism": "dp1", "hip_graph": bool(graphs), "optimizer": adam},
        "timing": {"regions_s": [round(r, 6) for r in regions], "reported": "median"},
        "loss_last_step": round(loss, 5), "finite": bool(np.isfinite(loss)),
    }
    if why:
        out["graph_capture_error"] = why
    out["roofline"] = ft_roofline(B)
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_ft(args.cpu_seconds, adversarial=False)
    print(json.dumps(_with_runtime(out)), flush=True)


def bench_adv_ft(args):
    """run_training's iteration with PointNetCls(k=40, feature_transform=True) as
    the generator.  Default: the fused feature-transform step run_training uses
    (step.AdvFtTrainStep: the generator's two batches as one C = 2B pass on the
    point-wise kernels, the plain step's tail for fc1 on, the hand-written
    extractor backward, both Adams in one launch), one HIP graph per resident
    batch pair.  --ft-body: the reference's body through autograd over the
    same kernels with capturable torch Adams (trainer._AutogradAdvStep, the
    path before round 6, run_training with args.fused_ft = False)."""
    import argparse
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd import trainer
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    from adversarial_learning_on_pointclouds_amd.step import AdvFtTrainStep
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = pc.PointNetCls(k=40, feature_transform=True).to(dev).train()
    model_D = pc.DeepConvDiscNet(40, 1).to(dev).train()
    pool = []
    for k in range(POOL):
        rng = np.random.default_rng(3500 + k)
        pool.append((torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev),
                     torch.from_numpy(rng.integers(0, 40, B)).to(dev),
                     torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev)))
    graphs, why = [], None
    if not args.ft_body:
        opts = [torch.optim.Adam(m.parameters(), lr=1e-4, betas=(0.9, 0.999))
                for m in (model, model_D)]
        adam = "fused (pcadv_adam2: both networks in one launch)"
        step = AdvFtTrainStep(model, model_D, B, N, optimizer=opts[0], optimizer_D=opts[1],
                              seed=1234, device=dev)
        if not args.no_graph:
            graphs = [step.capture_on(*p) for p in pool]
        workload = ("run_training iteration with PointNetCls(k=40, feature_transform=True) + "
                    "DeepConvDiscNet(40, 1): fused feature-transform step (AdvFtTrainStep)")
    else:
        opts = []
        for m in (model, model_D):
            try:
                opts.append(torch.optim.Adam(m.parameters(), lr=1e-4, betas=(0.9, 0.999),
                                             fused=True, capturable=True))
                adam = "torch.optim.Adam(fused=True, capturable=True)"
            except (RuntimeError, ValueError):
                opts.append(torch.optim.Adam(m.parameters(), lr=1e-4, betas=(0.9, 0.999),
                                             capturable=True))
                adam = "torch.optim.Adam(capturable=True)"
        targs = argparse.Namespace(device=str(dev), lambda_cls=1.0, lambda_adv=0.001)
        step = trainer._AutogradAdvStep(model, model_D, opts[0], opts[1],
                                        torch.nn.BCEWithLogitsLoss(), torch.nn.CrossEntropyLoss(),
                                        (ImagePool(0), ImagePool(0)), targs, B, N)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # autograd / optimizer state created outside any capture
            for k in range(3):
                step(*pool[k % POOL])
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if not args.no_graph:
            try:
                kept = []  # each graph's gradient buffers (the next capture drops p.grad)
                for k in range(POOL):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        step(*pool[k])
                    graphs.append(g)
                    kept.append([p.grad for p in list(model.parameters()) +
                                 list(model_D.parameters())])
            except Exception as e:  # noqa: BLE001 - reported in the line, eager timing instead
                graphs, why = [], f"{type(e).__name__}: {e}"[:200]
                torch.cuda.synchronize()
        workload = ("run_training iteration with PointNetCls(k=40, feature_transform=True) + "
                    "DeepConvDiscNet(40, 1): autograd body over the pcadv ops, two Adams")

    def one(k):
        if graphs:
            graphs[k % POOL].replay()
        else:
            step(*pool[k % POOL])
    for k in range(args.warmup):
        one(k)
    regions = timed_regions(one, args.steps, args.repeats)
    dt = float(np.median(regions))
    vals = [float(v) for v in step.losses[:4].cpu()]
    out = {
        "metric": "point-clouds/sec (adversarial train step, generator with feature_transform=True), "
                  "B=32+32 N=1024 ModelNet40, 1 GPU",
        "value": round(2 * B * args.steps / dt, 1), "unit": "clouds/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "fp32 (point-wise layers exact-f32 MFMA, 1024-channel conv + max as split "
                 "products with the exact max re-evaluated, head / D f32)",
        "data": "synthetic (seeded U(-1,1) clouds, labels in [0,40); resident in HBM)",
        "config": {"workload": workload, "global_batch": 2 * B, "points": N,
                   "parallelism": "dp1", "hip_graph": bool(graphs), "optimizer": adam},
        "timing": {"regions_s": [round(r, 6) for r in regions], "reported": "median"},
        "losses_last_step": [round(v, 5) for v in vals],
        "finite": bool(np.all(np.isfinite(vals))),
    }
    if why:
        out["graph_capture_error"] = why
    # the dominant kernel: the 1024-channel conv + max, twice per generator pass
    # (over the 2B clouds of both batches in the fused step, B in the body)
    C = B if args.ft_body else 2 * B
    roof = ft_roofline(C)
    if not args.ft_body:
        roof["traffic"], roof["traffic_source"] = _pmc_traffic(
            "r*_adv_ft_pmc_traffic.json", ["pcadv::k_conv4_max"])
        roof["traffic_unit"] = "bytes/launch (L2->memory, PMC FETCH_SIZEx2+WRITE_SIZE)"
        roof["mfma_busy"], roof["mfma_busy_source"] = _pmc_mfma("adv_ft", "k_conv4_max")
    out["roofline"] = roof
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_ft(args.cpu_seconds, adversarial=True)
    print(json.dumps(_with_runtime(out)), flush=True)


def _synthetic_modelnet(n_gt, n_nogt, seed=5000):
    """ModelNetDatasetGT / _noGT objects over in-memory synthetic clouds (the
    HDF5 files are not in the image): same attributes as the file-backed ones,
    data_augmentation on (the reference default, dataset/modelNetData.py:19)."""
    from adversarial_learning_on_pointclouds_amd import dataset as D
    rng = np.random.default_rng(seed)
    gt = D.ModelNetDatasetGT.__new__(D.ModelNetDatasetGT)
    gt.sample_list, gt.npoints, gt.data_augmentation = None, N, True
    gt.select_data = rng.uniform(-1, 1, (n_gt, N, 3)).astype(np.float32)
    gt.select_labels = rng.integers(0, 40, n_gt).astype(np.int32)
    ng = D.ModelNetDataset_noGT.__new__(D.ModelNetDataset_noGT)
    ng.sample_list, ng.npoints, ng.data_augmentation = None, N, True
    ng.select_data = rng.uniform(-1, 1, (n_nogt, N, 3)).astype(np.float32)
    return gt, ng


def bench_trainer(args):
    """The drop-in loop a user of the reference calls: trainer.run_training
    (utils/trainer.py:403-608) over two DeviceCloudLoaders (GT / no-GT split
    resident in HBM, each batch gathered and jittered on the device), B=32 +
    32, N=1024, loss lines logged every iteration (read asynchronously).
    Steady state = (T(W + K) - T(W)) / K over two fresh runs (iteration 0's
    test pass, checkpoint and graph capture cancel), median of --repeats."""
    import argparse as ap_
    import logging
    import tempfile
    from adversarial_learning_on_pointclouds_amd import dataset as D
    from adversarial_learning_on_pointclouds_amd import trainer
    from adversarial_learning_on_pointclouds_amd.image_pool import ImagePool
    dev = torch.device("cuda", 0)
    gt_ds, ng_ds = _synthetic_modelnet(1024, 4096)
    log = logging.getLogger("bench_trainer")
    log.addHandler(logging.NullHandler())
    log.propagate = False

    def run(iters, use_graph):
        model, model_D = make_models(dev, seed=0)
        opt = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999))
        opt_D = torch.optim.Adam(model_D.parameters(), lr=1e-4, betas=(0.9, 0.999))
        gt = D.DeviceCloudLoader(gt_ds, B, seed=1, drop_last=True)
        ng = D.DeviceCloudLoader(ng_ds, B, seed=2, drop_last=True)
        te = [next(iter(gt))]
        a = ap_.Namespace(device="cuda", total_iterations=iters, iter_save_epoch=10 ** 9,
                          iter_test_epoch=10 ** 9, exp_dir=tempfile.mkdtemp(prefix="bench_tr_"),
                          tensorboard=False, lambda_cls=1.0, lambda_adv=0.001, batch_size=B,
                          use_graph=use_graph, log_every=1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        trainer.run_training(gt, ng, enumerate(gt), enumerate(ng), te, model, model_D,
                             torch.nn.BCEWithLogitsLoss(), torch.nn.CrossEntropyLoss(), opt, opt_D,
                             ImagePool(0), ImagePool(0), log, log, None, a)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    W, K = args.warmup, args.steps
    run(W, True)  # first-use costs (library load, allocator) out of the timed runs
    per, per_eager = [], []
    for _ in range(args.repeats):
        per.append((run(W + K, True) - run(W, True)) / K)
    for _ in range(max(1, args.repeats // 3)):
        per_eager.append((run(W + K, False) - run(W, False)) / K)
    dt = float(np.median(per))
    # the graph-replay step over resident batches (the headline bench's timed loop)
    model, model_D = make_models(dev, seed=0)
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
    step = AdvTrainStep(model, model_D, B, N, seed=1234, device=dev)
    rng = np.random.default_rng(1000)
    bufs = (torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev),
            torch.from_numpy(rng.integers(0, 40, B)).to(dev),
            torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev))
    g = step.capture_on(*bufs)
    for _ in range(W):
        g.replay()
    reg = timed_regions(lambda k: g.replay(), K, args.repeats)
    replay = float(np.median(reg)) / K
    out = {
        "metric": "point-clouds/sec (run_training over DeviceCloudLoader, adv step), B=32 N=1024, 1 GPU",
        "value": round(2 * B / dt, 1), "unit": "clouds/s", "n_gpus": 1, "steps": K, "warmup": W,
        "ms_per_step": round(dt * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32 (f32-level, as the headline line)",
        "data": "synthetic in-memory ModelNet-shaped split (1024 GT + 4096 no-GT clouds), resident "
                "in HBM, device gather + jitter per batch",
        "config": {"workload": "trainer.run_training (utils/trainer.py:403-608) fed by two "
                               "DeviceCloudLoaders, loss lines every iteration (async)",
                   "global_batch": 2 * B, "points": N, "parallelism": "dp1",
                   "hip_graph": "gathers + fused step, one graph per iteration"},
        "timing": {"per_step_s": [round(v, 7) for v in per],
                   "method": "(T(W+K) - T(W)) / K of whole run_training calls, median"},
        "eager_ms_per_step": round(float(np.median(per_eager)) * 1e3, 4),
        "graph_replay_ms_per_step": round(replay * 1e3, 4),
        "ratio_to_graph_replay": round(dt / replay, 4),
    }
    print(json.dumps(_with_runtime(out)), flush=True)


def bench_seg(args):
    """BASELINE.json configs[3]: PointNetSeg ShapeNet-part B=16, N=2048, one
    run_training_pointnet_seg iteration (forward, per-point CE, backward, Adam)
    per step, HIP-graph replayed over resident synthetic batches."""
    import adversarial_learning_on_pointclouds_amd as pc
    from adversarial_learning_on_pointclouds_amd.seg import SegTrainStep
    from adversarial_learning_on_pointclouds_amd.model_utils import init_weights
    Bs, Ns = 16, 2048
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    # fp32 (the reference's dtype, six-product GEMMs) unless --precision bf16:
    # the labelled bf16x3 speed option (three-product forward / data gradients)
    precision = "bf16x3" if args.precision == "bf16" else "fp32"
    model = pc.PointNetSeg(50, precision=precision).to(dev)
    init_weights(model, "xavier", verbose=False)
    step = SegTrainStep(model, device=dev)
    pool = []
    for k in range(2):
        rng = np.random.default_rng(2000 + k)
        cls = np.zeros((Bs, 1, 16), np.float32)
        cls[np.arange(Bs), 0, rng.integers(0, 16, Bs)] = 1
        pool.append((torch.from_numpy(rng.uniform(-1, 1, (Bs, Ns, 3)).astype(np.float32)).to(dev),
                     torch.from_numpy(cls).to(dev),
                     torch.from_numpy(rng.integers(0, 50, (Bs, Ns))).to(dev)))
    graphs = [step.capture_on(*b) for b in pool]
    for k in range(args.warmup):
        graphs[k % 2].replay()
    regions = timed_regions(lambda k: graphs[k % 2].replay(), args.steps, args.repeats)
    dt = float(np.median(regions))
    # algorithmic FLOPs per step (fc1's tiled part once per cloud;
    # sparse max backward): forward 2 N (3*64 + 64*128 + 2*128*128 + 128*512 +
    # 512*2048 + 960*256 + 256*256 + 256*128 + 128*50) per cloud, backward twice
    # the dense layers except conv6 (sparse) and conv1's input gradient
    per_pt_fwd = 3 * 64 + 64 * 128 + 2 * 128 * 128 + 128 * 512 + 512 * 2048 + 960 * 256 + \
        256 * 256 + 256 * 128 + 128 * 50
    dense_bwd = 2 * (per_pt_fwd - 512 * 2048) - 3 * 64
    gflop = 2.0 * Bs * Ns * (per_pt_fwd + dense_bwd) / 1e9
    loss = float(step.loss.item())
    # dominant kernel: conv6 + ReLU + max over points as the step runs it
    # (pcadv_conv_max_bf2: the screened GEMM k_gemm_bf2_big<2> (256x256 tiles) on the bf16 planes
    # conv5's epilogue wrote + the exact re-evaluation k_max_combine), timed with
    # HIP events on the current stream over the last batch's x5
    from adversarial_learning_on_pointclouds_amd import seg as segmod
    from adversarial_learning_on_pointclouds_amd._lib import check, stream_ptr
    import ctypes
    params = [p for p in model.parameters()]
    segmod._engine().split(step.param, step.wph, step.wpl)
    fw = segmod.seg_forward(pool[(args.steps - 1) % 2][0], pool[(args.steps - 1) % 2][1], params,
                            wplanes=step.wplanes, precision=precision)
    lib = segmod._engine().lib
    gmax = torch.empty(Bs, 2048, device=dev)
    gidx = torch.empty(Bs, 2048, device=dev, dtype=torch.int32)
    wsb = lib.pcadv_conv_max_x3_workspace_bytes(Bs, Ns, 2048)
    ws = torch.empty(wsb, device=dev, dtype=torch.uint8)
    W6 = fw["W"][5]
    b6 = params[11]
    x5 = ctypes.c_void_p(fw["xloc"].data_ptr() + 4 * segmod._OFF[4])

    x5p, w6p = fw["x5p"], fw["W6p"]
    big = os.environ.get("PCADV_GEMM_BIG", "1") != "0"
    glds = os.environ.get("PCADV_GEMM_GLDS", "1") != "0"
    gname = (f"k_gemm_bf2_big<2, {'true' if glds else 'false'}> (operands staged by "
             f"{'LDS-DMA' if glds else 'registers'})") if big else "k_gemm_x3<2,2,2,3>"
    kname = f"pcadv_conv_max_bf2: {gname}" if x5p is not None else "pcadv_conv_max_x3: k_gemm_x3<0,0,2,3>"

    def cmx():
        if x5p is not None:
            (hi, lo), ld, off = x5p
            check(lib.pcadv_conv_max_bf2(x5, segmod._LOC, segmod._pb(hi, off), segmod._pb(lo, off),
                                         ld, Bs, Ns, 512,
                                         ctypes.c_void_p(W6.data_ptr()), segmod._pb(w6p[0]),
                                         segmod._pb(w6p[1]), ctypes.c_void_p(b6.data_ptr()), 2048, 1,
                                         ctypes.c_void_p(gmax.data_ptr()), ctypes.c_void_p(gidx.data_ptr()),
                                         ctypes.c_void_p(ws.data_ptr()), wsb, stream_ptr()), "conv_max_bf2")
            return
        check(lib.pcadv_conv_max_x3(x5, segmod._LOC, Bs, Ns, 512, ctypes.c_void_p(W6.data_ptr()),
                                    ctypes.c_void_p(b6.data_ptr()), 2048, 1,
                                    ctypes.c_void_p(gmax.data_ptr()), ctypes.c_void_p(gidx.data_ptr()),
                                    ctypes.c_void_p(ws.data_ptr()), wsb, stream_ptr()), "conv_max_x3")
    for _ in range(3):
        cmx()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    ev0.record()
    for _ in range(reps):
        cmx()
    ev1.record()
    torch.cuda.synchronize()
    kern_s = ev0.elapsed_time(ev1) / 1e3 / reps
    kflops = 2.0 * Bs * Ns * 512 * 2048
    kissued = 3 * kflops  # three bf16 MFMA products per f32 product (hi/lo splits)
    busy, busy_src = _pmc_mfma("seg", "k_gemm_bf2_big<2" if big else "k_gemm_x3<2, 2, 2, 3>") \
        if precision == "fp32" else (None, None)
    traffic, traffic_src = _pmc_traffic(
        "r*_seg_pmc_traffic.json",
        ("pcadv::k_gemm_bf2_big<2" if big else "pcadv::k_gemm_x3<2, 2, 2, 3>", "pcadv::k_max_combine"))
    out = {
        "metric": "point-clouds/sec (seg train step), B=16 N=2048 ShapeNet-part, 1 GPU",
        "value": round(Bs * args.steps / dt, 1), "unit": "clouds/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": ("fp32 (f32-level: every GEMM as six bf16 hi/mid/lo MFMA products, f32 "
                  "accumulate; conv6's max screened with three products and every winner "
                  "re-evaluated in exact f32)") if precision == "fp32" else
                 ("bf16x3 (below fp32, a labelled speed option: forward and data-gradient GEMMs "
                  "as three bf16 hi/lo MFMA products, f32 accumulate; weight gradients six "
                  "products)"),
        "data": "synthetic (seeded U(-1,1) clouds, one-hot classes, part labels in [0,50))",
        "config": {"workload": "PointNetSeg(50) + CrossEntropyLoss + Adam, B=16, N=2048 "
                               "(BASELINE configs[3])", "global_batch": Bs, "points": Ns,
                   "parallelism": "dp1", "hip_graph": True},
        "timing": {"regions_s": [round(r, 6) for r in regions], "reported": "median"},
        "roofline": {"bound": "mfma",
                     "kernel": kname + " (conv6 512->2048 screened top-2 per 128-point tile) "
                               "+ k_max_combine (exact f32 re-evaluation)",
                     "achieved": round(kflops / kern_s / 1e12, 2), "peak": BF16_PEAK,
                     "unit": "TFLOP/s", "frac": round(kflops / kern_s / 1e12 / BF16_PEAK, 4),
                     "issued_frac": round(kissued / kern_s / 1e12 / BF16_PEAK, 4),
                     "traffic": traffic,
                     "traffic_unit": "bytes/launch (L2->memory, PMC FETCH_SIZEx2+WRITE_SIZE)",
                     "traffic_source": traffic_src, "avg_launch_us": round(kern_s * 1e6, 2),
                     "mfma_busy": busy, "mfma_busy_source": busy_src,
                     "algorithmic_flops_per_launch": kflops,
                     "algorithmic_bytes_per_launch": Bs * Ns * 512 * 4 + 2048 * 512 * 4 + Bs * 2048 * 8,
                     "issued_bf16_flops_per_launch": kissued,
                     "peak_basis": "dense bf16 MFMA 2500 TF, the pipe the kernel runs on; achieved = "
                                   "algorithmic f32 FLOPs / launch time (issued_frac: the three "
                                   "bf16 split products per f32 product)"},
        "step_flops": {"gflop_per_step": round(gflop, 2),
                       "achieved_tflops": round(gflop * args.steps / dt / 1e3, 2)},
        "loss_last_step": round(loss, 5), "finite": bool(np.isfinite(loss)),
    }
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_seg(args.cpu_seconds, Bs, Ns)
    print(json.dumps(_with_runtime(out)), flush=True)


def bench_dp1(args):
    """what the data-parallel iteration costs beyond the
    step itself, on the one GPU there is.  A one-rank RCCL group (the
    all-reduce's average is then the identity, so every form computes the
    plain step bitwise, tests/test_gpu_distributed.py) times, over the same
    resident batches and alternating in one process:
      plain   the step's HIP graph (bench.py's headline form);
      dp4     DataParallelAdvStep.capture: four graphs (step part 1 | part 2 |
              Adam of the early bucket | Adam of conv1..conv4) around the two
              host-issued RCCL all-reduces (bench --gpus N, trainer _DPIteration);
      dp1g    DataParallelAdvStep.capture_single: the same iteration as ONE graph
              with both all-reduces captured on RCCL's stream;
      dp2     overlap=False: the step without Adam | ONE all-reduce of the 4.2 MB
              gradient buffer | both Adams (two graphs around one collective);
      dp2g    the same as ONE graph with the all-reduce captured - the default
              since round 6 (DataParallelAdvStep.graphed on RCCL: bench --gpus N,
              trainer _DPIteration), and the line's value.
    overhead = form - plain per iteration (the communication itself is ~0 on
    one rank; the multi-rank exchange is the driver's scaling runs)."""
    import torch.distributed as tdist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    tdist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
    from adversarial_learning_on_pointclouds_amd.distributed import DataParallelAdvStep
    model, model_D = make_models(dev, seed=0)
    step = AdvTrainStep(model, model_D, B, N, seed=1234, device=dev, precision="fp32")
    runner = DataParallelAdvStep(step, overlap=True)
    flat = DataParallelAdvStep(step, broadcast_params=False, overlap=False)
    pool = []
    for k in range(POOL):
        rng = np.random.default_rng(1000 + k * 64)
        pool.append((torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev),
                     torch.from_numpy(rng.integers(0, 40, B)).to(dev),
                     torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev)))
    forms = {"plain": [step.capture_on(*p) for p in pool],
             "dp4": [runner.capture(*p) for p in pool],
             "dp2": [flat.capture(*p) for p in pool]}
    single_err = None
    for name, r in (("dp1g", runner), ("dp2g", flat)):
        try:
            forms[name] = [r.capture_single(*p) for p in pool]
        except Exception as e:  # noqa: BLE001 - reported in the line
            single_err = f"{name}: {type(e).__name__}: {e}"[:300]
    host = {}
    times = {k: [] for k in forms}
    for _ in range(args.repeats):
        for name, gs in forms.items():
            for k in range(args.warmup):
                gs[k % POOL].replay()
            t_enq = []
            def one(k, gs=gs):
                t0 = time.perf_counter()
                gs[k % POOL].replay()
                t_enq.append(time.perf_counter() - t0)
            times[name] += timed_regions(one, args.steps, 1)
            host[name] = float(np.median(t_enq)) * 1e6
    ms = {k: float(np.median(v)) / args.steps * 1e3 for k, v in times.items()}
    out = {
        "metric": "data-parallel iteration overhead on a one-rank RCCL group (adv step, B=32+32, N=1024)",
        "value": round((ms["dp2g"] - ms["plain"]) * 1e3, 2) if "dp2g" in ms else None,
        "unit": "us/iteration (default form dp2g - plain)",
        "higher_is_better": False, "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": {k: round(v, 4) for k, v in ms.items()},
        "overhead_us": {k: round((v - ms["plain"]) * 1e3, 2) for k, v in ms.items() if k != "plain"},
        "host_enqueue_us_per_iteration": {k: round(v, 1) for k, v in host.items()},
        "regions_s": {k: [round(r, 6) for r in v] for k, v in times.items()},
        "single_graph_capture_error": single_err,
        "note": "forms alternated per repeat in one process; one rank: the all-reduce averages "
                "nothing, so this is the iteration's structure cost (graph splits, host-issued "
                "collectives, stream waits), not xGMI time",
    }
    print(json.dumps(_with_runtime(out)), flush=True)
    tdist.destroy_process_group()


def main():
    global N
    args = parse()
    N = args.points
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if args.config != "adv":
            raise SystemExit(f"--config {args.config} is a single-GPU workload; --gpus applies to adv")
        return spawn_ranks(args.gpus)  # no GPU call has been made in this process
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks: "
                         "refusing to report a different n_gpus")
    if args.launch_check:
        return launch_check(args, world, rank)
    if args.config == "seg":
        return bench_seg(args)
    if args.config == "cls":
        return bench_cls(args)
    if args.config == "cls_ft":
        return bench_cls_ft(args)
    if args.config == "adv_ft":
        return bench_adv_ft(args)
    if args.config == "trainer":
        return bench_trainer(args)
    if args.config == "dp1":
        return bench_dp1(args)
    if _backend() != "nccl":  # rehearsal: ranks may share a GPU
        local %= max(1, torch.cuda.device_count())
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as tdist
        backend = _backend()
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=dev)
        else:
            tdist.init_process_group(backend)
        dist = tdist
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)

    from adversarial_learning_on_pointclouds_amd import ops
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
    from adversarial_learning_on_pointclouds_amd.distributed import DataParallelAdvStep

    model, model_D = make_models(dev, seed=0)
    adv_prec = args.precision or "fp32"
    # DataParallelAdvStep keys the device draws by global rows (rank 0's seed)
    step = AdvTrainStep(model, model_D, B, N, seed=1234, device=dev, precision=adv_prec)
    # PCADV_BENCH_OVERLAP=1 selects the round-5 bucketed, overlapped all-reduce
    overlap = os.environ.get("PCADV_BENCH_OVERLAP", "") == "1"
    runner = DataParallelAdvStep(step, overlap=overlap) if dist is not None else None

    # resident synthetic inputs: rank-specific shards of the global batch
    pool = []
    for k in range(POOL):
        rng = np.random.default_rng(1000 + k * 64 + rank)
        pool.append((torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev),
                     torch.from_numpy(rng.integers(0, 40, B)).to(dev),
                     torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev)))
    use_graph = not args.no_graph
    graphs = []
    G = 1
    seq = None
    if use_graph:
        if runner is not None:  # over RCCL one graph per iteration, all-reduce captured
            graphs = [runner.graphed(*pool[k]) for k in range(POOL)]
        else:
            graphs = [step.capture_on(*pool[k]) for k in range(POOL)]
            G = max(1, min(args.graph_steps, POOL))
            seq = step.capture_seq(pool[:G]) if G > 1 else None
    run = graph_runner(graphs, seq, G)

    def one(k, total):
        if use_graph:
            run(k, total)
        elif runner is not None:
            runner(*pool[k % POOL])
        else:
            step(*pool[k % POOL])

    for k in range(args.warmup):
        one(k, args.warmup)
    regions = timed_regions(lambda k: one(k, args.steps), args.steps, args.repeats, dist)
    dt = float(np.median(regions))
    losses = step.losses[:4].cpu().numpy().tolist()
    finite = all(np.isfinite(losses))

    # dominant kernel k_conv4_max and the feature forward pair, timed with HIP
    # events over the last resident batch (the step's 2B clouds)
    pg, lab, pn = pool[(args.steps - 1) % POOL]
    pts_all = torch.cat([pg, pn], 0).contiguous()
    fw = [model.feat.conv1.weight, model.feat.conv1.bias, model.feat.conv2.weight,
          model.feat.conv2.bias, model.feat.conv3.weight, model.feat.conv3.bias,
          model.feat.conv4.weight, model.feat.conv4.bias]
    # the committed PMC passes ran the default workload (fp32, N = 1024)
    roof = feat_roofline(pts_all, fw, adv_prec,
                         "r*_pmc_traffic.json" if (N == 1024 and adv_prec == "fp32") else None,
                         "adv" if (N == 1024 and adv_prec == "fp32") else None)
    pair = roof["pair"]
    # algorithmic FLOPs of one B=32 adversarial step (44.53 at N=2048)
    step_gflop = 22.47 if N == 1024 else 22.47 * N / 1024.0
    step_tf = step_gflop * world * args.steps / dt / 1e3

    result = {
        "metric": f"point-clouds/sec (adv train step), B=32 N={N} ModelNet40, 1/2/4/8 GPU",
        "value": round(2 * B * args.steps * world / dt, 1),
        "unit": "clouds/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("fp32 (f32-level: conv3/conv4 as bf16 split-product MFMAs, f32 accumulate, "
                  "each max winner re-evaluated in exact f32)" if adv_prec == "fp32" else
                  "bf16 (conv3 / conv4 MFMAs on bf16-rounded operands, f32 accumulate; the rest f32)"),
        "data": "synthetic (seeded U(-1,1) clouds, labels in [0,40); resident in HBM)",
        "config": {"workload": "adversarial cls step: PointNetCls(k=40)+DeepConvDiscNet(40,1), "
                               f"B=32 GT + 32 noGT clouds/GPU, N={N}, Adam x2",
                   "global_batch": 2 * B * world, "points": N,
                   "parallelism": f"dp{world}", "hip_graph": use_graph, "steps_per_graph": G,
                   **({"dp_iteration": runner.graph_form} if runner is not None else {})},
        "world_size": world,
        "backend": ((_backend() if _backend() != "nccl" else "nccl (RCCL)") if world > 1 else None),
        "timing": {"regions_s": [round(r, 6) for r in regions], "reported": "median",
                   "per_region": "barrier + synchronize on both sides, max over ranks"},
        "roofline": roof,
        "fp32_equivalent": {
            "kernel": "feature forward pair (conv1..conv4 + max)",
            "achieved_tflops": pair["achieved"], "f32_mfma_peak_tflops": F32_PEAK,
            "note": "algorithmic f32 FLOPs / time against the f32 MFMA peak; the f32 products are "
                    "emulated on the bf16 pipe (split operands, f32 accumulate, winners "
                    "re-evaluated in exact f32), so this is not a roofline fraction"},
        "step_flops": {"gflop_per_step": step_gflop, "achieved_tflops": round(step_tf, 2)},
        "losses_last_step": [round(v, 5) for v in losses],
        "finite": finite,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(_with_runtime(result)), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
