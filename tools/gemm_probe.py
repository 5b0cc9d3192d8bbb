"""Times single seg GEMM launches through the C ABI (HIP events, median of
20): fc1's data gradient (32 768 x 960 x 256, W^T, output mask) with and
without its mask, fc1's weight gradient (six products over 32 768 rows), and
the two as one paired launch.  Diagnostic only (outputs are not checked)."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from adversarial_learning_on_pointclouds_amd import _lib  # noqa: E402
from adversarial_learning_on_pointclouds_amd._lib import check, stream_ptr  # noqa: E402


def _p(t, off=0):
    return ctypes.c_void_p(t.data_ptr() + 4 * off)


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    M, B, N = 32768, 16, 2048
    dh1 = torch.randn(M, 256, device=dev)
    W1 = torch.randn(256, 3024, device=dev)
    xloc = torch.randn(M, 960, device=dev)
    dloc = torch.empty(M, 960, device=dev)
    dW1 = torch.empty(256, 3024, device=dev)
    db1 = torch.empty(256, device=dev)
    s1 = torch.empty(B, 256, device=dev)
    nb = lib.pcadv_gemm_wgrad_workspace_bytes(M, 256, 960, N)
    ws = torch.empty(nb, device=dev, dtype=torch.uint8)

    def dgrad(mask=True):
        check(lib.pcadv_gemm(_p(dh1), 256, 0, _p(W1), 3024, 1, _p(dloc), 960, M, 960, 256, None, None,
                             0, 0, 0, _p(xloc) if mask else None, 960 if mask else 0, 0, None, None, 0,
                             stream_ptr()), "dgrad")

    def wgrad():
        check(lib.pcadv_gemm_wgrad(_p(dh1), 256, _p(xloc), 960, M, 256, 960, _p(dW1), 3024, _p(db1),
                                   _p(s1), N, 0, _p(ws), nb, stream_ptr()), "wgrad")

    def pair():
        check(lib.pcadv_gemm_pair_begin(stream_ptr()), "begin")
        dgrad()
        wgrad()
        check(lib.pcadv_gemm_pair_end(stream_ptr()), "end")

    for name, fn in (("dgrad masked", lambda: dgrad(True)), ("dgrad no mask", lambda: dgrad(False)),
                     ("wgrad (+ finish)", wgrad), ("pair (+ finish)", pair)):
        print(f"PROBE {name:18s} {timed(fn):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
