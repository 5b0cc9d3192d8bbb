"""Block-level timeline of the adversarial step's head/discriminator chain
(fc1 .. the last k_linear_bwd) inside a replayed HIP graph (diagnostic build:
`make stamps` -> build/stamps/libpcadv_stamps.so, never the product library).

Per launch: first and last block start, the median block's 'tile summed' and
'partials met' stamps (wave 0), the last block end; and the gap from the
previous launch's last end to this launch's first start (the in-kernel view of
a launch boundary).  s_memrealtime ticks at 100 MHz (10 ns).

    python tools/lin_stamps.py [B] [N]
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

LIN_NAMES = ("fc1 fwd", "fc2 fwd", "D conv2 fwd", "D conv3 fwd", "D conv3 bwd", "D conv2 bwd",
             "fc2 bwd", "fc1 bwd")
TAIL = (("k_head_fwd", lambda B: (2 * B + 15) // 16), ("k_disc_tail", lambda B: (3 * B + 15) // 16),
        ("k_head_bwd", lambda B: (2 * B + 15) // 16))


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    lib = _lib.load()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = pc.PointNetCls(k=40).to(dev)
    model_D = pc.DeepConvDiscNet(40, 1).to(dev)
    step = pc.AdvTrainStep(model, model_D, B, N, device=dev)
    g = torch.Generator().manual_seed(1)
    pts_gt = (torch.rand(B, N, 3, generator=g) * 2 - 1).to(dev)
    pts_nogt = (torch.rand(B, N, 3, generator=g) * 2 - 1).to(dev)
    labels = torch.randint(0, 40, (B,), generator=g).to(dev)
    for _ in range(3):
        step(pts_gt, labels, pts_nogt)
    torch.cuda.synchronize()
    rd = lib.pcadv_lin_stamps
    rd.restype = ctypes.c_int
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert rd(None, 1) == 0
    st = step.capture()  # eager warm-up takes slots 0..7, the captured launches 8..15
    st[0].copy_(pts_gt)
    st[1].copy_(labels)
    st[2].copy_(pts_nogt)
    for _ in range(20):
        step.replay()
    torch.cuda.synchronize()
    host = (ctypes.c_uint64 * (16 * 256 * 6))()
    assert rd(host, 0) == 0
    lin = np.frombuffer(host, dtype=np.uint64).astype(np.int64).reshape(16, 256, 6)
    th = (ctypes.c_uint64 * (3 * 16 * 16))()
    f = lib.pcadv_tail_stamps
    f.restype = ctypes.c_int
    assert f(th) == 0
    tail = np.frombuffer(th, dtype=np.uint64).astype(np.int64).reshape(3, 16, 16)

    rows = []
    for i, name in enumerate(LIN_NAMES):
        s = lin[8 + i]
        used = s[:, 0] > 0
        s = s[used]
        mid = s[:, 1] > 0
        iss = np.median(s[mid, 5] - s[mid, 0]) * 10 / 1e3 if mid.any() else np.nan
        name = f"{name} [issue {iss:.2f}]"
        rows.append((s[:, 0].min(), s[:, 0].max(), np.median(s[mid, 4]) if mid.any() else np.nan,
                     np.median(s[mid, 1]) if mid.any() else np.nan,
                     np.median(s[mid, 2]) if mid.any() else np.nan, s[:, 3].max(),
                     f"{name} ({used.sum()} blocks)"))
    for k, (name, nb) in enumerate(TAIL):
        s = tail[k, :nb(B)]
        cols = [c for c in range(16) if (s[:, c] > 0).all()]
        rows.append((s[:, 0].min(), s[:, 0].max(), np.nan, np.nan, np.nan, s[:, cols[-1]].max(),
                     f"{name} ({nb(B)} blocks, end = last stamp)"))
    rows.sort(key=lambda r: r[0])
    t0 = rows[0][0]
    us = lambda t: (t - t0) * 10 / 1e3  # noqa: E731
    print("first_start last_start  landed_med  tile_med  met_med  last_end   span   gap_before  launch")
    prev_end = None
    for r in rows:
        gap = "" if prev_end is None else f"{(r[0] - prev_end) * 10 / 1e3:6.2f}"
        print(f"{us(r[0]):10.2f} {us(r[1]):10.2f} {us(r[2]):11.2f} {us(r[3]):9.2f} {us(r[4]):8.2f} "
              f"{us(r[5]):9.2f} {(r[5] - r[0]) * 10 / 1e3:6.2f}   {gap:>8}    {r[6]}")
        prev_end = r[5]


if __name__ == "__main__":
    main()
