"""Calibrate the CPU baseline (container only: imports the reference from
/root/reference, which never travels to the GPU box).

Times the reference's own run_training (utils/trainer.py:403-608) at B=32,
N=1024 on this host's cores, steady state = (T(K2) - T(K1)) / (K2 - K1)
(iteration 0 also saves a checkpoint and runs the test pass), and the numpy
oracle's adversarial step on the same shapes, so DESIGN.md can state how far
the port used as bench.py's cpu_baseline is from the reference.

    python tools/time_reference_cpu.py [/root/reference] [--out profiles/rNN_cpu_calibration.json]
"""
import argparse
import logging
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import pointnet_np as onp  # noqa: E402

B, N = 32, 1024


def time_reference(ref_root, iters):
    sys.dont_write_bytecode = True
    sys.path.insert(0, ref_root)
    import torch
    import torch.nn as nn
    from models.pointnet import PointNetCls
    from models.discriminator import DeepConvDiscNet
    import utils.trainer as rtrainer
    from utils.image_pool import ImagePool

    torch.set_num_threads(os.cpu_count())
    rng = np.random.default_rng(1000)
    gt = [(torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)),
           torch.from_numpy(rng.integers(0, 40, B).astype(np.int64))) for _ in range(iters)]
    ng = [torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)) for _ in range(iters)]
    model, model_D = PointNetCls(k=40), DeepConvDiscNet(40, 1)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    opt_D = torch.optim.Adam(model_D.parameters(), lr=1e-4)
    log = logging.getLogger("calib")
    log.addHandler(logging.NullHandler())
    log.propagate = False
    args = argparse.Namespace(device=torch.device("cpu"), total_iterations=iters, lambda_cls=1.0,
                              lambda_adv=0.001, iter_save_epoch=10 ** 9, iter_test_epoch=10 ** 9,
                              exp_dir=tempfile.mkdtemp(prefix="calib_"), tensorboard=False,
                              batch_size=B)
    t0 = time.perf_counter()
    rtrainer.run_training(trainloader_gt=gt, trainloader_nogt=ng,
                          trainloader_gt_iter=enumerate(list(gt)),
                          targetloader_nogt_iter=enumerate(list(ng)), testloader=gt[:1],
                          model=model, model_D=model_D, gan_loss=nn.BCEWithLogitsLoss(),
                          cls_loss=nn.CrossEntropyLoss(), optimizer=opt, optimizer_D=opt_D,
                          history_pool_gt=ImagePool(0), history_pool_nogt=ImagePool(0),
                          train_logger=log, test_logger=log, writer=None, args=args)
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ref_root", nargs="?", default="/root/reference")
    ap.add_argument("--rounds", type=int, default=3, help="alternating reference / port timings")
    ap.add_argument("--out", default=None, help="write the summary JSON here (e.g. profiles/)")
    a = ap.parse_args()
    import json
    import bench
    k1, k2 = 3, 13
    refs, ports, dense = [], [], []
    for _ in range(a.rounds):  # alternate, so host drift hits all alike
        t1, t2 = time_reference(a.ref_root, k1), time_reference(a.ref_root, k2)
        refs.append(2 * B * (k2 - k1) / (t2 - t1))
        st, dt = bench._time_adv_oracle(10.0, dense=False)
        ports.append(2 * B * st / dt)
        st, dt = bench._time_adv_oracle(10.0, dense=True)
        dense.append(2 * B * st / dt)
    ref_v, port_v, dense_v = float(np.median(refs)), float(np.median(ports)), float(np.median(dense))
    out = {"cores": os.cpu_count(), "threads": "torch.set_num_threads(cores); numpy/BLAS default",
           "reference_run_training_clouds_per_s": round(ref_v, 1),
           "reference_ms_per_step": round(2 * B / ref_v * 1e3, 1),
           "port_clouds_per_s": round(port_v, 1), "port_over_reference": round(port_v / ref_v, 3),
           "dense_port_clouds_per_s": round(dense_v, 1),
           "dense_port_over_reference": round(dense_v / ref_v, 3),
           "samples": {"reference": [round(v, 1) for v in refs], "port": [round(v, 1) for v in ports],
                       "dense_port": [round(v, 1) for v in dense]},
           "workload": "adversarial step B=32 GT + 32 no-GT, N=1024, fp32 (run_training :426-559)",
           "method": "reference: (T(13) - T(3)) / 10 iterations of utils/trainer.py:run_training "
                     "(iteration 0's checkpoint + test pass cancel); port / dense_port: "
                     "bench._time_adv_oracle(10 s) with the sparse / the reference's dense max-pool "
                     "backward (bench.py's cpu_baseline times the dense one); "
                     f"median of {a.rounds} alternating rounds"}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
