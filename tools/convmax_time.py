"""Time the conv + max backward (k_convmax_bwd) alone, with and without the
data gradient, at the feature-transform path's shapes (C clouds x N points,
K = 128 -> O = 1024).

    python tools/convmax_time.py [C] [N]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from adversarial_learning_on_pointclouds_amd import ops  # noqa: E402


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.relu(torch.randn(C, N, 128, generator=g)).to(dev)
    w = (torch.randn(1024, 128, generator=g) / 12).to(dev)
    b = torch.zeros(1024).to(dev)
    gmax, gidx = ops.conv_max_fwd(x, w, b, False)
    dg = torch.randn(C, 1024, generator=g).to(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for need_dx in (False, True):
        for _ in range(5):
            ops.conv_max_bwd(dg, gidx, x, w, None, need_dx)
        e0.record()
        for _ in range(50):
            ops.conv_max_bwd(dg, gidx, x, w, None, need_dx)
        e1.record()
        torch.cuda.synchronize()
        print(f"conv_max_bwd C={C} N={N} need_dx={need_dx}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us")


if __name__ == "__main__":
    main()
