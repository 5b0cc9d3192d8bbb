"""Calibrate the CPU baseline (container only: imports the reference from
/root/reference, which never travels to the GPU box).

Times the reference's own run_training (utils/trainer.py:403-608) at B=32,
N=1024 on this host's cores, steady state = (T(K2) - T(K1)) / (K2 - K1)
(iteration 0 also saves a checkpoint and runs the test pass), and the numpy
oracle's adversarial step on the same shapes, so DESIGN.md can state how far
the port used as bench.py's cpu_baseline is from the reference.

    python tools/time_reference_cpu.py [/root/reference]
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
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    k1, k2 = 3, 13
    t1, t2 = time_reference(ref, k1), time_reference(ref, k2)
    ref_step = (t2 - t1) / (k2 - k1)
    import bench
    port = bench.cpu_baseline(15.0)
    print(f"cores={os.cpu_count()}")
    print(f"reference run_training: {ref_step * 1e3:.1f} ms/step = {2 * B / ref_step:.1f} clouds/s")
    print(f"numpy oracle port:      {port['value']:.1f} clouds/s ({port['sample']})")
    print(f"port / reference = {port['value'] / (2 * B / ref_step):.3f}")


if __name__ == "__main__":
    main()
