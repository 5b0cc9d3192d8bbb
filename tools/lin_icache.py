"""Is a small launch's start slow because of its first instruction fetches?
(diagnostic build: `make stamps`).  Launches the fc1 backward shape
(M = 64, N = 512, K = 1024, data + weight gradients) through pcadv_linear_bwd:

  cold: a 256 MiB copy between launches evicts L2 and instruction caches
  warm: the same launch three times back to back

and prints each launch's median 'loads issued' and 'operands landed' times
after the block's first stamp (s_memrealtime, 10 ns ticks).

    python tools/lin_icache.py
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PCADV_LIB"] = os.environ.get("PCADV_STAMPS_LIB", os.path.join(REPO, "build", "stamps", "libpcadv_stamps.so"))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from adversarial_learning_on_pointclouds_amd import _lib  # noqa: E402


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    M, N, K = 64, 512, 1024
    g = torch.Generator(device="cpu").manual_seed(0)
    dy = torch.randn(M, N, generator=g).to(dev)
    x = torch.randn(M, K, generator=g).to(dev)
    w = torch.randn(N, K, generator=g).to(dev)
    dx = torch.empty(M, K, device=dev)
    dw = torch.empty(N, K, device=dev)
    db = torch.empty(N, device=dev)
    big_a = torch.empty(64 << 20, device=dev)
    big_b = torch.empty(64 << 20, device=dev)
    rd = lib.pcadv_lin_stamps
    rd.restype = ctypes.c_int
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
    f = lib.pcadv_linear_bwd
    f.restype = ctypes.c_int
    P = ctypes.c_void_p

    def launch():
        rc = f(P(dy.data_ptr()), None, 0, None, None, ctypes.c_uint64(0), ctypes.c_float(0.0),
               P(x.data_ptr()), P(w.data_ptr()), P(dx.data_ptr()), P(dw.data_ptr()),
               P(db.data_ptr()), M, M, N, K, P(torch.cuda.current_stream().cuda_stream))
        assert rc == 0

    launch()
    torch.cuda.synchronize()
    assert rd(None, 1) == 0
    labels = []
    for i in range(3):  # cold: evict between launches
        big_b.copy_(big_a)
        launch()
        labels.append("cold")
    for i in range(3):  # warm: back to back
        launch()
        labels.append("warm")
    torch.cuda.synchronize()
    host = (ctypes.c_uint64 * (16 * 256 * 6))()
    assert rd(host, 0) == 0
    st = np.frombuffer(host, dtype=np.uint64).astype(np.int64).reshape(16, 256, 6)
    for i, lab in enumerate(labels):
        s = st[i]
        s = s[(s[:, 0] > 0) & (s[:, 5] > 0)]
        iss = np.median(s[:, 5] - s[:, 0]) * 10 / 1e3
        land = np.median(s[:, 4] - s[:, 0]) * 10 / 1e3
        tile = np.median(s[:, 1] - s[:, 0]) * 10 / 1e3
        print(f"{lab}: {len(s)} data blocks  issued {iss:5.2f} us  landed {land:5.2f} us  "
              f"tile {tile:5.2f} us")


if __name__ == "__main__":
    main()
