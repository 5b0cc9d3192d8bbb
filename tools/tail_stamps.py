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
    # the chunk_prepare halves (hit sort + active-row records) riding in
    # k_disc_tail / k_cls_head: [half][0 start, 1 sorted, 2 loads, 3 conv1,
    # 4 conv2 MFMA, 5 x2 stored, 6 x1 stored] (thread 0 of each half)
    if hasattr(lib, "pcadv_prep_stamps"):
        hp = (ctypes.c_uint64 * (1024 * 8))()
        assert lib.pcadv_prep_stamps(hp) == 0
        ps = np.frombuffer(hp, dtype=np.uint64).astype(np.int64).reshape(1024, 8)
        ps = ps[ps[:, 0] > 0]
        t0 = ps[:, 0].min()
        print(f"== chunk_prepare: {ps.shape[0]} halves; starts spread {(ps[:, 0].max() - t0) * 10 / 1e3:.2f} us")
        for a, b, nm in ((0, 1, "sort"), (1, 2, "pts/W loads"), (2, 3, "conv1"), (3, 4, "conv2 MFMA"),
                         (4, 5, "x2 stores"), (5, 6, "masks")):
            m = (ps[:, a] > 0) & (ps[:, b] > 0)
            if m.any():
                d = (ps[m, b] - ps[m, a]) * 10 / 1e3
                print(f"  {nm:12s} median {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f} us")
        last = np.where(ps[:, 6] > 0, ps[:, 6], ps[:, 1])
        print(f"  last end {(last.max() - t0) * 10 / 1e3:.2f} us after the first start")
    # the in-step chunk launch (k_feat_bwd_chunk<true>): chunk workgroups carry
    # nact in slot 15, trailing (dW4 gather / Adam) workgroups -1
    if hasattr(lib, "pcadv_chunk_stamps"):
        hc = (ctypes.c_uint64 * (1024 * 32))()
        assert lib.pcadv_chunk_stamps(hc) == 0
        cs = np.frombuffer(hc, dtype=np.uint64).astype(np.int64).reshape(1024, 32)
        used = cs[:, 0] > 0
        cs = cs[used]
        tr = cs[:, 15] < 0
        ch = cs[~tr]
        t0 = cs[:, 0].min()
        us = lambda v: (v - t0) * 10 / 1e3
        nact = ch[:, 15]
        print(f"== k_feat_bwd_chunk<true> in the step: {ch.shape[0]} chunks, {int(tr.sum())} trailing")
        print(f"  chunk end max {us(ch[:, 14]).max():.2f} us; trailing start min {us(cs[tr, 0]).min():.2f} "
              f"median {np.median(us(cs[tr, 0])):.2f}, end max {us(cs[tr, 14]).max():.2f}")
        for code, nm in ((-1, "dW4 gather"), (-2, "Adam")):
            m = cs[:, 15] == code
            if m.any():
                d = (cs[m, 14] - cs[m, 0]) * 10 / 1e3
                print(f"  {nm:10s} {int(m.sum()):3d} workgroups: start median {np.median(us(cs[m, 0])):.2f} "
                      f"span median {np.median(d):.2f} max {d.max():.2f}, end max {us(cs[m, 14]).max():.2f}")
        span = (ch[:, 14] - ch[:, 0]) * 10 / 1e3
        for lo, hi in ((0, 32), (33, 64), (65, 128)):
            m = (nact >= lo) & (nact <= hi)
            if m.any():
                print(f"  nact {lo:3d}-{hi:3d}: {int(m.sum()):4d} chunks, span median {np.median(span[m]):.2f} "
                      f"max {span[m].max():.2f}, end max {us(ch[m, 14]).max():.2f} us")
        names = ["setup", "", "", "a", "b+combine", "c dX2", "d dX1", "e wgrad"]
        for nm, a, b in (("setup", 0, 3), ("a", 3, 4), ("b+combine", 4, 5), ("c dX2", 5, 6),
                         ("d dX1", 6, 7), ("e wgrad", 7, 8)):
            d = (ch[:, b] - ch[:, a]) * 10 / 1e3
            print(f"  batch1 {nm:10s} median {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f}")
        # diagnostic sub-stamps of batch 1 (thread 0): phase a 24..26, phase c 28..30
        for nm, a, b in (("a: start", 3, 24), ("a: conv1", 24, 25), ("a: conv2+W2 wait", 25, 26),
                         ("a: epilogue", 26, 4), ("c: B loads", 5, 28), ("c: MFMA", 28, 29),
                         ("c: park+barrier", 29, 30), ("c: combine", 30, 6)):
            ok = (ch[:, a] > 0) & (ch[:, b] > 0)
            if ok.any():
                d = (ch[ok, b] - ch[ok, a]) * 10 / 1e3
                print(f"    {nm:16s} median {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f}")
        two = nact > 32
        if two.any():
            for nm, a, b in (("a", 8, 9), ("b+combine", 9, 10), ("c dX2", 10, 11), ("d dX1", 11, 12),
                             ("e wgrad", 12, 13)):
                d = (ch[two, b] - ch[two, a]) * 10 / 1e3
                print(f"  batch2 {nm:10s} median {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f}")


if __name__ == "__main__":
    main()
