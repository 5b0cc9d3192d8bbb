"""Run the PointNetfeat forward (and backward) a few times on the product
library: a short, quiet program for rocprofv3 kernel-trace / PMC passes.

    python tools/feat_fwd_run.py [reps] [C] [N]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from adversarial_learning_on_pointclouds_amd import ops  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    pts = (torch.rand(C, N, 3, generator=g) * 2 - 1).to(dev)

    def u(*s, fan):
        return ((torch.rand(*s, generator=g) * 2 - 1) / fan ** 0.5).to(dev)
    w = [u(64, 3, fan=3), u(64, fan=3), u(64, 64, fan=64), u(64, fan=64), u(128, 64, fan=64),
         u(128, fan=64), u(1024, 128, fan=128), u(1024, fan=128)]
    dg = torch.randn(C, 1024, device=dev) * 1e-3
    for _ in range(reps):
        gmax, gidx, x3 = ops.feat_fwd(pts, *w)
        ops.feat_bwd(dg, gidx, pts, w[0], w[1], w[2], w[3], w[4], w[6], x3)
    torch.cuda.synchronize()
    print("ok", float(gmax.sum()))


if __name__ == "__main__":
    main()
