"""Dump pcadv_feat_fwd outputs (x3, gmax, gidx) for seeded inputs, for a
bitwise comparison of two library builds (PCADV_LIB):

    PCADV_LIB=build/ab/libA.so python tools/featfwd_dump.py A
    python tools/featfwd_dump.py B
    python tools/featfwd_dump.py --compare A B
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.path.join(REPO, "gpurun_out")
CASES = [(64, 1024), (3, 1000), (5, 77), (64, 2048)]


def dump(tag):
    import torch
    from adversarial_learning_on_pointclouds_amd import ops
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(7)
    w = [(torch.rand(*s, generator=g) * 2 - 1) / f ** 0.5 for s, f in
         [((64, 3), 3), ((64,), 3), ((64, 64), 64), ((64,), 64), ((128, 64), 64), ((128,), 64),
          ((1024, 128), 128), ((1024,), 128)]]
    w = [t.to(dev) for t in w]
    for C, N in CASES:
        pts = (torch.rand(C, N, 3, generator=g) * 2 - 1).to(dev)
        for prec in ("fp32", "bf16"):
            gmax, gidx, x3 = ops.feat_fwd(pts, *w, precision=prec)
            np.savez(os.path.join(OUT, f"ffd_{tag}_{C}_{N}_{prec}.npz"), gmax=gmax.cpu().numpy(),
                     gidx=gidx.cpu().numpy(), x3=x3.cpu().numpy())
    print("dumped", tag)


def compare(a, b):
    ok = True
    for C, N in CASES:
        for prec in ("fp32", "bf16"):
            A = np.load(os.path.join(OUT, f"ffd_{a}_{C}_{N}_{prec}.npz"))
            B = np.load(os.path.join(OUT, f"ffd_{b}_{C}_{N}_{prec}.npz"))
            same = all(np.array_equal(A[k].view(np.uint32) if A[k].dtype == np.float32 else A[k],
                                      B[k].view(np.uint32) if B[k].dtype == np.float32 else B[k])
                       for k in ("x3", "gmax", "gidx"))
            print(f"C={C} N={N} {prec}: {'bitwise equal' if same else 'DIFFERENT'}")
            ok &= same
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        dump(sys.argv[1])
