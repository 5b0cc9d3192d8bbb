"""Per-tensor comparison of the HIP PointNetSeg step with the numpy oracle
(diagnostics for tests/test_gpu_seg.py)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import pointnet_np as onp  # noqa: E402
from adversarial_learning_on_pointclouds_amd.seg import PointNetSeg, seg_cross_entropy  # noqa: E402


def main():
    S = onp.make_params(onp.seg_spec(50), seed=21)
    rng = np.random.default_rng(22)
    B, N = 3, 700
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    cls = np.zeros((B, 1, 16), np.float32)
    cls[np.arange(B), 0, rng.integers(0, 16, B)] = 1
    seg = rng.integers(0, 50, (B, N))
    m = PointNetSeg(50)
    m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in S.items()})
    m = m.cuda()
    t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).cuda().to(dt)
    logits, g, gi = m.forward_points(t(pts), t(cls))
    loss = seg_cross_entropy(logits, t(seg, torch.int64))
    loss.backward()
    rl, grads, rlog, rg, ram = onp.seg_step(S, pts, cls, seg)
    print("loss", loss.item(), rl)
    e = lambda a, r: float(np.abs(a - r).max() / max(np.abs(r).max(), 1e-30))
    print("logits", e(logits.detach().cpu().numpy(), rlog), "gmax", e(g.detach().cpu().numpy(), rg))
    gi = gi.cpu().numpy()
    print("argmax mismatches", int((gi != ram).sum()), "of", gi.size, "(positive)",
          int(((gi != ram) & (rg > 0)).sum()))
    for name, p in m.named_parameters():
        print(f"{name:14s} {e(p.grad.cpu().numpy(), grads[name]):.3e}")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def fp64_grads(S, pts, cls, seg):
    """float64 torch autograd of the same network: the arbiter."""
    B, N, _ = pts.shape
    T = {k: torch.tensor(v, dtype=torch.float64, device="cuda", requires_grad=True) for k, v in S.items()}
    x = torch.tensor(pts, dtype=torch.float64, device="cuda")
    xs = []
    h = x
    for i in range(1, 7):
        h = torch.relu(h @ T[f"conv{i}.weight"][:, :, 0].T + T[f"conv{i}.bias"])
        xs.append(h)
    gm = xs[5].max(1).values
    c = torch.tensor(cls, dtype=torch.float64, device="cuda")
    feat = torch.cat(xs[:5] + [gm[:, None, :].expand(B, N, 2048), c.expand(B, N, 16)], 2)
    h = torch.relu(feat @ T["fc1.weight"].T + T["fc1.bias"])
    h = torch.relu(h @ T["fc2.weight"].T + T["fc2.bias"])
    h = torch.relu(h @ T["fc3.weight"].T + T["fc3.bias"])
    o = h @ T["fc4.weight"].T + T["fc4.bias"]
    l = torch.nn.functional.cross_entropy(o.permute(0, 2, 1), torch.tensor(seg, device="cuda"))
    l.backward()
    return {k: T[k].grad.cpu().numpy() for k in S}


def main2():
    S = onp.make_params(onp.seg_spec(50), seed=21)
    rng = np.random.default_rng(22)
    B, N = 3, 700
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    cls = np.zeros((B, 1, 16), np.float32)
    cls[np.arange(B), 0, rng.integers(0, 16, B)] = 1
    seg = rng.integers(0, 50, (B, N))
    ref = fp64_grads(S, pts, cls, seg)
    _, og, _, _, _ = onp.seg_step(S, pts, cls, seg)
    m = PointNetSeg(50)
    m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in S.items()})
    m = m.cuda()
    t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).cuda().to(dt)
    lg, _, _ = m.forward_points(t(pts), t(cls))
    seg_cross_entropy(lg, t(seg, torch.int64)).backward()
    e = lambda a, r: float(np.abs(a - r).max() / max(np.abs(r).max(), 1e-30))
    print("param          oracle-vs-fp64  hip-vs-fp64")
    for name, p in m.named_parameters():
        print(f"{name:14s} {e(og[name], ref[name]):.3e}       {e(p.grad.cpu().numpy(), ref[name]):.3e}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "fp64":
    main2()


def main3():
    os.environ["PCADV_SEG_DEBUG"] = "1"
    import importlib
    import adversarial_learning_on_pointclouds_amd.seg as segm
    importlib.reload(segm)
    S = onp.make_params(onp.seg_spec(50), seed=21)
    rng = np.random.default_rng(22)
    B, N = 3, 700
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    cls = np.zeros((B, 1, 16), np.float32)
    cls[np.arange(B), 0, rng.integers(0, 16, B)] = 1
    seg = rng.integers(0, 50, (B, N))
    m = segm.PointNetSeg(50)
    m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in S.items()})
    m = m.cuda()
    t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).cuda().to(dt)
    lg, _, _ = m.forward_points(t(pts), t(cls))
    segm.seg_cross_entropy(lg, t(seg, torch.int64)).backward()
    D = {k: v.double().cpu().numpy() for k, v in segm._DEBUG.items()}
    dh2 = (D["dh3"] * (D["h3"] > 0)) @ D["W3"]
    dh1 = (D["dh2"] * (D["h2"] > 0)) @ D["W2"]
    e = lambda a, r: float(np.abs(a - r).max() / max(np.abs(r).max(), 1e-30))
    print("dh2 vs own-input fp64:", e(D["dh2"], dh2), " dh1:", e(D["dh1"], dh1))
    bad = np.argwhere(np.abs(D["dh2"] - dh2) > 1e-3 * np.abs(dh2).max())
    print("bad dh2 entries", len(bad), bad[:10].tolist())
    rows = np.unique(bad[:, 0]) if len(bad) else []
    print("bad rows", len(rows), list(rows[:20]))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "dbg":
    main3()


def main4():
    os.environ["PCADV_SEG_DEBUG"] = "1"
    import importlib
    import adversarial_learning_on_pointclouds_amd.seg as segm
    importlib.reload(segm)
    S = onp.make_params(onp.seg_spec(50), seed=21)
    rng = np.random.default_rng(22)
    B, N = 3, 700
    pts = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    cls = np.zeros((B, 1, 16), np.float32)
    cls[np.arange(B), 0, rng.integers(0, 16, B)] = 1
    seg = rng.integers(0, 50, (B, N))
    m = segm.PointNetSeg(50)
    m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in S.items()})
    m = m.cuda()
    t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).cuda().to(dt)
    lg, _, _ = m.forward_points(t(pts), t(cls))
    segm.seg_cross_entropy(lg, t(seg, torch.int64)).backward()
    D = {k: v.double().cpu().numpy() for k, v in segm._DEBUG.items()}
    # fp64 forward with retained intermediates
    T = {k: torch.tensor(v, dtype=torch.float64, device="cuda", requires_grad=True) for k, v in S.items()}
    x = torch.tensor(pts, dtype=torch.float64, device="cuda")
    xs = []
    h = x
    for i in range(1, 7):
        h = torch.relu(h @ T[f"conv{i}.weight"][:, :, 0].T + T[f"conv{i}.bias"])
        xs.append(h)
    gm = xs[5].max(1).values
    c = torch.tensor(cls, dtype=torch.float64, device="cuda")
    feat = torch.cat(xs[:5] + [gm[:, None, :].expand(B, N, 2048), c.expand(B, N, 16)], 2)
    h1 = torch.relu(feat @ T["fc1.weight"].T + T["fc1.bias"]); h1.retain_grad()
    h2 = torch.relu(h1 @ T["fc2.weight"].T + T["fc2.bias"]); h2.retain_grad()
    h3 = torch.relu(h2 @ T["fc3.weight"].T + T["fc3.bias"]); h3.retain_grad()
    o = h3 @ T["fc4.weight"].T + T["fc4.bias"]; o.retain_grad()
    l = torch.nn.functional.cross_entropy(o.permute(0, 2, 1), torch.tensor(seg, device="cuda"))
    l.backward()
    R = dict(dl=o.grad, dh3=h3.grad, dh2=h2.grad, dh1=h1.grad, h1=h1, h2=h2, h3=h3)
    e = lambda a, r: float(np.abs(a - r).max() / max(np.abs(r).max(), 1e-30))
    for k in ["dl", "h3", "h2", "h1", "dh3", "dh2", "dh1"]:
        r = R[k].detach().reshape(B * N, -1).cpu().numpy()
        print(k, e(D[k], r), "zeros ours/ref", int((D[k] == 0).sum()), int((r == 0).sum()))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "cmp":
    main4()
