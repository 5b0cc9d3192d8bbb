"""What certifying k_conv4_max's argmax would have to re-check (VERDICT r05
item 2b), measured with the diagnostic library built with
-DPCADV_C4_CERT=2 (build/cert/libcert2.so; never loaded by the product):
every lane also tracks the largest screened key it drops, so after the exact
re-evaluation of the top two each channel knows its third screened value v3,
and it is counted when v3 + bound reaches the winner's exact value, i.e. when
a dropped point could still be the true maximum:

  rigorous   bound = 2^-14 ||x||max ||w_o||  (the screening error's worst case,
             see the kernel comment: three dropped split terms, 384 f32
             accumulation roundings, the 2^-17 key truncation, Cauchy-Schwarz)
  empirical  bound = 2^-17 ||x||max ||w_o||  (about 2x the largest screening
             error measured, 4.4e-6 sum|x w|)

on (a) the bench's adversarial step (configs[2]: 64 clouds per step), (b) the
near-tie stress clouds of tools/diag_argmax.py.  Counts per launch of the
64-cloud conv4 (65 536 channels).

    PCADV_LIB=build/cert/libcert2.so python tools/cert_diag.py [out.json]
"""
import ctypes
import json
import os
import sys

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from adversarial_learning_on_pointclouds_amd import _lib, ops  # noqa: E402


def read(lib):
    buf = (ctypes.c_uint * 4)()
    torch.cuda.synchronize()
    if lib.pcadv_c4_cert_read(buf) != 0:
        raise RuntimeError("pcadv_c4_cert_read failed")
    return list(buf)


def per_launch(c):
    n = max(1, c[3])
    return {"launches": c[3], "channels": c[1], "flagged_rigorous": c[0],
            "flagged_empirical": c[2],
            "rigorous_per_launch": round(c[0] / n, 2), "empirical_per_launch": round(c[2] / n, 2),
            "rigorous_frac": c[0] / max(1, c[1]), "empirical_frac": c[2] / max(1, c[1])}


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    lib = _lib.load()
    if not hasattr(lib, "pcadv_c4_cert_read"):
        raise SystemExit("set PCADV_LIB to a -DPCADV_C4_CERT=2 build (build/cert/libcert2.so)")
    lib.pcadv_c4_cert_read.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from adversarial_learning_on_pointclouds_amd.step import AdvTrainStep
    model, model_D = bench.make_models(dev, seed=0)
    B, N = bench.B, bench.N
    step = AdvTrainStep(model, model_D, B, N, seed=1234, device=dev)
    pool = []
    for k in range(bench.POOL):
        rng = np.random.default_rng(1000 + k * 64)
        pool.append((torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev),
                     torch.from_numpy(rng.integers(0, 40, B)).to(dev),
                     torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)).to(dev)))
    graphs = [step.capture_on(*p) for p in pool]
    for k in range(5):
        graphs[k % len(graphs)].replay()
    read(lib)
    for k in range(40):  # 40 training steps: the weights move, the data cycles
        graphs[k % len(graphs)].replay()
    res = {"adv_step_40_steps": per_launch(read(lib))}
    # the stress clouds of tools/diag_argmax.py (near-duplicate points, maxima near 0)
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from oracle import pointnet_np as onp
    stress = {}
    for ws, tw in ((1.0, 0.0), (64.0, 3e-6), (8.0, 1e-5), (1.0, 1e-6), (64.0, 3e-7)):
        C = 24
        G = onp.make_params(onp.cls_spec(40), seed=41)
        G["feat.conv4.weight"] = (G["feat.conv4.weight"] * np.float32(ws)).astype(np.float32)
        base = np.random.default_rng(42).uniform(-1, 1, (1, N, 3)).astype(np.float32)
        if tw:
            base[:, 1::2] = base[:, 0::2] + np.random.default_rng(44).normal(0, tw, base[:, 0::2].shape)
        pts = (base + np.random.default_rng(43).normal(0, 1e-4, (C, N, 3))).astype(np.float32)
        if tw:
            pts[:, 1::2] = pts[:, 0::2] + (base[:, 1::2] - base[:, 0::2])
        _, _, x3 = onp.point_mlp_fwd(pts, G)
        W4 = G["feat.conv4.weight"][:, :, 0].astype(np.float64)
        m = np.stack([(x3[c].astype(np.float64) @ W4.T).max(0) for c in range(C)])
        G["feat.conv4.bias"] = (-m.mean(0)).astype(np.float32)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
        w = [t(G[n]) for n in ["feat.conv1.weight", "feat.conv1.bias", "feat.conv2.weight",
                               "feat.conv2.bias", "feat.conv3.weight", "feat.conv3.bias",
                               "feat.conv4.weight", "feat.conv4.bias"]]
        ops.feat_fwd(t(pts), *w)
        stress[f"w_scale={ws} twin={tw}"] = per_launch(read(lib))
    res["stress_24_clouds"] = stress
    s = json.dumps(res, indent=1)
    print(s, flush=True)
    if out_path:
        with open(out_path, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
