"""Time the feature forward pair and k_conv4_max alone (HIP events over a
graph of 50 back-to-back launches) on the library PCADV_LIB points at: the
A/B harness of k_conv4_max variants.

    PCADV_LIB=... python tools/k2_time.py [C] [N] [precision]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from adversarial_learning_on_pointclouds_amd import ops  # noqa: E402


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    prec = sys.argv[3] if len(sys.argv) > 3 else "fp32"
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    pts = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, (C, N, 3)).astype(np.float32)).to(dev)

    def u(*s, fan):
        return ((torch.rand(*s) * 2 - 1) / fan ** 0.5).to(dev)
    fw = [u(64, 3, 1, fan=3), u(64, fan=3), u(64, 64, 1, fan=64), u(64, fan=64), u(128, 64, 1, fan=64),
          u(128, fan=64), u(1024, 128, 1, fan=128), u(1024, fan=128)]
    gmax, gidx, x3 = ops.feat_fwd(pts, *fw, precision=prec)
    pair = bench._graph_time(lambda: ops.feat_fwd(pts, *fw, precision=prec))
    k2 = bench._graph_time(lambda: ops.conv4_max(x3, fw[6], fw[7], precision=prec, out=(gmax, gidx)))
    print(f"pair_us {pair * 1e6:.2f} k2_us {k2 * 1e6:.2f}")


if __name__ == "__main__":
    main()
