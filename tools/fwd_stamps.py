"""Per-phase timestamps of the fused feature forward / backward (diagnostic
build: `make stamps` -> build/stamps/libpcadv_stamps.so, never the product
library).  s_memrealtime ticks at 100 MHz (10 ns).

    python tools/fwd_stamps.py [C] [N]
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
from adversarial_learning_on_pointclouds_amd._lib import stream_ptr  # noqa: E402


def summarize(tag, st, cols):
    st = st.astype(np.int64)
    t0 = st[:, 0].min()
    rel = (st - t0) * 10 / 1e3  # us
    print(f"== {tag}: {st.shape[0]} workgroups; first start 0, last start "
          f"{rel[:, 0].max():.2f} us, last end {max(rel[:, c].max() for c in cols[-1:]):.2f} us")
    prev = 0
    for c in cols:
        d = (st[:, c] - st[:, prev]) * 10 / 1e3
        print(f"  stamp {prev:2d}->{c:2d}: median {np.median(d):7.2f} us  p10 {np.percentile(d, 10):7.2f}"
              f"  p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f}")
        prev = c


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    lib = _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    pts = (torch.rand(C, N, 3, generator=g) * 2 - 1).to(dev)
    def u(*s, fan):
        return ((torch.rand(*s, generator=g) * 2 - 1) / fan ** 0.5).to(dev)
    w1, b1 = u(64, 3, fan=3), u(64, fan=3)
    w2, b2 = u(64, 64, fan=64), u(64, fan=64)
    w3, b3 = u(128, 64, fan=64), u(128, fan=64)
    w4, b4 = u(1024, 128, fan=128), u(1024, fan=128)
    x3 = torch.empty(C, N, 128, device=dev)
    gmax = torch.empty(C, 1024, device=dev)
    gidx = torch.empty(C, 1024, device=dev, dtype=torch.int32)
    nb = lib.pcadv_feat_fwd_workspace_bytes(C, N)
    ws = torch.empty(nb, device=dev, dtype=torch.uint8)
    T = (N + 127) // 128
    stamps = torch.zeros(C * ((T + 1) // 2) * 16 + C * T * 16, device=dev, dtype=torch.int64)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    f = lib.pcadv_feat_fwd_stamped
    f.restype = ctypes.c_int
    args = [P(pts), C, N, P(w1), P(b1), P(w2), P(b2), P(w3), P(b3), P(w4), P(b4), P(x3), P(gmax),
            P(gidx), P(ws), ctypes.c_size_t(nb), P(stamps), stream_ptr()]
    for _ in range(5):
        assert f(*args) == 0
    torch.cuda.synchronize()
    nwg = C * 4
    st = stamps[:nwg * 16].view(nwg, 16).cpu().numpy()
    # k_conv4_max thread 0: 0 start, 1 W4 + first tile staged, 2 point loop done, 3 end
    # 6 + j: end of step 2 j + 1 (every other 64-point step, up to 8 of them)
    S = (N + 63) // 64
    steps = [6 + j for j in range(min(8, S // 2))]
    summarize("k_conv4_max", st, [1] + steps + [2, 4, 5, 3])
    n1 = (C * ((N + 63) // 64) + 1) // 2
    st1 = stamps[nwg * 16:nwg * 16 + n1 * 16].view(n1, 16).cpu().numpy()
    st1 = st1[st1[:, 0] > 0]
    ntiles = C * ((N + 63) // 64)
    if st1.shape[0] < n1:
        # k_point_mlp_ws (one workgroup per CU): 1 weights split; 3 + it after the
        # barrier of pipeline step it (A: tile it, B: tile it - 1); 2 end
        tpw = (ntiles + 255) // 256
        summarize("k_point_mlp_ws", st1, [1] + [3 + i for i in range(min(tpw + 1, 13))] + [2])
    else:
        # k_point_mlp thread 0: 1 weights loaded; per tile t: 3+5t pts staged, 4+5t conv1,
        # 5+5t conv2 (+split), 6+5t conv3 MFMAs, 7+5t x3 stores issued; 2 both tiles done
        summarize("k_point_mlp", st1, [1, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 2])
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(20):
        f(*args)
    ev1.record()
    torch.cuda.synchronize()
    print(f"  feat_fwd (k_point_mlp + k_conv4_max) event time: {ev0.elapsed_time(ev1) / 20 * 1e3:.2f} us")

    dg = torch.randn(C, 1024, device=dev) * 1e-3
    grads = [torch.empty_like(t) for t in (w1, b1, w2, b2, w3, b3, w4, b4)]
    nbb = lib.pcadv_feat_bwd_workspace_bytes(C, N)
    wsb = torch.empty(nbb, device=dev, dtype=torch.uint8)
    sb = torch.zeros(C * T * 32, device=dev, dtype=torch.int64)
    fb = lib.pcadv_feat_bwd_stamped
    fb.restype = ctypes.c_int
    bargs = [P(dg), P(gidx), P(pts), C, N, P(w1), P(b1), P(w2), P(b2), P(w3), P(w4), P(x3)] + \
            [P(t) for t in grads] + [P(wsb), ctypes.c_size_t(nbb), P(sb), stream_ptr()]
    for _ in range(5):
        assert fb(*bargs) == 0
    torch.cuda.synchronize()
    sbw = sb.view(C * T, 32).cpu().numpy().astype(np.int64)
    sbn = sbw[:, :16]
    cols = [c for c in range(1, 15) if (sbn[:, c] > 0).all()]
    summarize("k_feat_bwd_chunk thread 0", sbn, cols)
    nact = sbn[:, 15]
    print("  active rows per chunk: median", np.median(nact), "max", nact.max(),
          "chunks > 32:", int((nact > 32).sum()), "of", len(nact))
    # stamps: 0 start, 1 hits, 2 compact, 3 sorted; batch k: 4+5k a(x1/x2), 5+5k b(dZ3),
    # 6+5k c(dX2), 7+5k d(dX1), 8+5k e(wgrad); 14 end
    t0 = sbn[:, 0].min()
    tot = (sbn[:, 14] - sbn[:, 0]) * 10 / 1e3
    end = (sbn[:, 14] - t0) * 10 / 1e3
    print(f"  workgroup span: median {np.median(tot):.2f} max {tot.max():.2f}; kernel end "
          f"{end.max():.2f} us after the first start")
    for lo, hi in ((0, 32), (33, 64), (65, 128)):
        m = (nact >= lo) & (nact <= hi)
        if m.any():
            print(f"  nact {lo:3d}-{hi:3d}: {int(m.sum()):4d} chunks, span median "
                  f"{np.median(tot[m]):.2f} max {tot[m].max():.2f} us")
    names = ["setup(hits)", "compact", "sort", "a x1/x2", "b dZ3", "c dX2", "d dX1", "e wgrad"]
    prev_cols = [0, 1, 2, 3, 4, 5, 6, 7]
    cur_cols = [1, 2, 3, 4, 5, 6, 7, 8]
    for nm, a, b in zip(names, prev_cols, cur_cols):
        d = (sbn[:, b] - sbn[:, a]) * 10 / 1e3
        print(f"  batch1 {nm:12s} median {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f}")
    d = (sbw[:, 16] - sbn[:, 3]) * 10 / 1e3
    print(f"  batch1 gather (wave 2, from the sort) median {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f}")
    for nm, a_, b_ in (("a: pts staged", 3, 24), ("a: conv1", 24, 25), ("a: conv2 MFMA", 25, 26),
                       ("a: x2 written", 26, 4)):
        ca = sbn[:, a_] if a_ < 16 else sbw[:, a_]
        cb = sbn[:, b_] if b_ < 16 else sbw[:, b_]
        d = (cb - ca) * 10 / 1e3
        print(f"  batch1 {nm:14s} median {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f}")
    two = nact > 32
    if two.any():
        for nm, a, b in zip(names[3:], [8, 9, 10, 11, 12], [9, 10, 11, 12, 13]):
            d = (sbn[two, b] - sbn[two, a]) * 10 / 1e3
            print(f"  batch2 {nm:12s} median {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f}")
        d = (sbn[two, 14] - sbn[two, 13]) * 10 / 1e3
        print(f"  slab write (2 batches) median {np.median(d):6.2f}")
    d = (sbn[~two, 14] - sbn[~two, 8]) * 10 / 1e3
    print(f"  slab write (1 batch) median {np.median(d):6.2f}")
    ev0.record()
    for _ in range(20):
        fb(*bargs)
    ev1.record()
    torch.cuda.synchronize()
    print(f"  feat_bwd (chunk + finish) event time: {ev0.elapsed_time(ev1) / 20 * 1e3:.2f} us")


if __name__ == "__main__":
    main()
