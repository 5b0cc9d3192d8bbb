"""Per-phase timestamps of the fused tail kernels (k_head_fwd, k_disc_tail,
k_head_bwd) over one eager adversarial step (diagnostic build: `make stamps`
-> build/stamps/libpcadv_stamps.so, never the product library).
s_memrealtime ticks at 100 MHz (10 ns).

    python tools/tail_stamps.py [B] [N]
    python tools/tail_stamps.py cls [B] [N]   (k_cls_head, slot 0)
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PCADV_LIB"] = os.environ.get("PCADV_STAMPS_LIB", os.path.join(REPO, "build", "stamps", "libpcadv_stamps.so"))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import adversarial_learning_on_pointclouds_amd as pc  # noqa: E402
from adversarial_learning_on_pointclouds_amd import _lib  # noqa: E402

NAMES = ("k_head_fwd", "k_disc_tail", "k_head_bwd")
NBLK = {"k_head_fwd": lambda B: (2 * B + 15) // 16, "k_disc_tail": lambda B: (3 * B + 15) // 16,
        "k_head_bwd": lambda B: (2 * B + 15) // 16}


def main():
    args = sys.argv[1:]
    cls = bool(args) and args[0] == "cls"
    if cls:
        args = args[1:]
    B = int(args[0]) if len(args) > 0 else 32
    N = int(args[1]) if len(args) > 1 else 1024
    lib = _lib.load()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = pc.PointNetCls(k=40).to(dev)
    g = torch.Generator().manual_seed(1)
    pts_gt = (torch.rand(B, N, 3, generator=g) * 2 - 1).to(dev)
    pts_nogt = (torch.rand(B, N, 3, generator=g) * 2 - 1).to(dev)
    labels = torch.randint(0, 40, (B,), generator=g).to(dev)
    if cls:
        step = pc.step.ClsTrainStep(model, B, N, device=dev, precision="bf16")
        for _ in range(5):
            step(pts_gt, labels)
    else:
        model_D = pc.DeepConvDiscNet(40, 1).to(dev)
        step = pc.AdvTrainStep(model, model_D, B, N, device=dev)
        for _ in range(5):
            step(pts_gt, labels, pts_nogt)
    torch.cuda.synchronize()
    host = (ctypes.c_uint64 * (3 * 16 * 16))()
    f = lib.pcadv_tail_stamps
    f.restype = ctypes.c_int
    assert f(host) == 0
    st = np.frombuffer(host, dtype=np.uint64).astype(np.int64).reshape(3, 16, 16)
    names = ("k_cls_head",) if cls else NAMES
    for k, name in enumerate(names):
        nb = 1 if cls else NBLK[name](B)
        s = st[k, :nb]
        t0 = s[:, 0].min()
        cols = [c for c in range(1, 16) if (s[:, c] > 0).all()]
        print(f"== {name}: {nb} row blocks; block starts spread {(s[:, 0].max() - t0) * 10 / 1e3:.2f} us")
        prev = 0
        for c in cols:
            d = (s[:, c] - s[:, prev]) * 10 / 1e3
            print(f"  stamp {prev:2d}->{c:2d}: median {np.median(d):6.2f} us  max {d.max():6.2f}")
            prev = c
        print(f"  block 0 total {(s[0, cols[-1]] - s[0, 0]) * 10 / 1e3:.2f} us")


if __name__ == "__main__":
    main()
