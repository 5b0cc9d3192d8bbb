#!/usr/bin/env python3
"""Why a one-product (bf16 hi x hi) screen cannot feed k_conv4_max's exact
re-evaluation with a bounded candidate list, measured on
the bench's inputs: configs[2]'s synthetic clouds (U(-1,1), N = 1024) through
conv1..conv3 with default-init weights (the oracle's restatement,
oracle/pointnet_np.py; CPU, numpy).

For each conv4 channel o of each cloud: the points whose exact value lies
within t * sum_k |x_k w_k| of the channel max (t = the screening error a
product count leaves: ~2^-8 for one product, ~2^-16 for three), and the
candidate count of a certified band for one product, threshold
s_max - 2 c |x|max |w_o| (c = 2^-7 * 1.05, the worst-case error of bf16 hi x hi
with f32 accumulation, Cauchy-Schwarz bound), with the per-lane overflow rate
of a top-K register list (K = 2, 3) in k_conv4_max's accumulator layout.

    python tools/band_study.py [clouds]   -> profiles/r04_band_study.txt
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from oracle.pointnet_np import bf16_round, cls_spec, make_params, point_mlp_fwd  # noqa: E402

F32 = np.float32


def main(clouds=8):
    p = make_params(cls_spec(40), 0)
    rng = np.random.default_rng(1000)
    N = 1024
    pts = rng.uniform(-1, 1, (clouds, N, 3)).astype(F32)
    _, _, x3 = point_mlp_fwd(pts, p)
    w = p["feat.conv4.weight"].reshape(1024, 128).astype(np.float64)
    wb = bf16_round(w.astype(F32)).astype(np.float64)
    wn = np.linalg.norm(w, axis=1)
    c = 2.0 ** -7 * 1.05
    half = (np.arange(N) % 32 >> 2) & 1  # which lane half of a 32-point unit holds the row
    ts = [2.0 ** -e for e in (6, 7, 8, 9, 10, 12, 14, 16)]
    cnt = {t: [] for t in ts}
    band, ovf = [], {2: 0, 3: 0}
    spread, err1 = [], []
    for b in range(clouds):
        x = x3[b].astype(np.float64)
        v = x @ w.T
        S = np.abs(x) @ np.abs(w).T
        am = v.argmax(0)
        Smax = S[am, np.arange(1024)]
        spread.append((v.std(0) / Smax).mean())
        for t in ts:
            cnt[t].append((v >= (v.max(0) - t * Smax)[None, :]).sum(0))
        s1 = bf16_round(x.astype(F32)).astype(np.float64) @ wb.T
        err1.append((np.abs(s1 - v) / S).max())
        T = s1.max(0) - 2 * c * np.linalg.norm(x, axis=1).max() * wn
        inb = s1 >= T[None, :]
        band.append(inb.sum(0))
        n0 = (inb & (half[:, None] == 0)).sum(0)
        n1 = (inb & (half[:, None] == 1)).sum(0)
        for K in ovf:
            ovf[K] += int(((n0 >= K) | (n1 >= K)).sum())
    tot = clouds * 1024
    out = [f"conv4 channel statistics over {clouds} clouds x 1024 channels (configs[2] inputs)",
           f"std over points of a channel's values / sum|x w| at its max: {np.mean(spread):.4f}",
           f"one-product screen error, max over (point, channel) / sum|x w|: {max(err1):.2e}",
           "points within t * sum|x w| of the channel max:",
           "  t        mean   p99   max"]
    for t in ts:
        a = np.concatenate(cnt[t])
        out.append(f"  2^{int(np.log2(t)):<4d} {a.mean():6.2f} {np.percentile(a, 99):5.0f} {a.max():5d}")
    a = np.concatenate(band)
    out.append(f"certified one-product band (c = 2^-7 * 1.05, |x|max |w_o|): candidates mean "
               f"{a.mean():.1f}, p99 {np.percentile(a, 99):.0f}, max {a.max()}")
    for K, n in ovf.items():
        out.append(f"  top-{K} per lane overflows on {n} / {tot} channels ({100 * n / tot:.1f} %)")
    return "\n".join(out)




def two_product(clouds=8):
    """the two-product screens, each with its rigorous band.

    A (W4 hi only): s = (x_hi + x_lo) . w_hi; |v - s| <= |x_p| |w_o - w_hi| + acc.
    B (x3 hi only): s = x_hi . (w_hi + w_lo); |v - s| <= |x_p - x_hi| |w_o| + acc.
    acc = 2^-15 |x_p| |w_o| covers the dropped lo.lo term (2^-16 relative) and
    the f32 accumulation of 128 products.  A point p can be channel o's argmax
    only if s_p + e_p >= max_q (s_q - e_q); the uniform form uses e = max_p e_p.
    The kernel keeps a top-K list per lane (two lanes per channel, each half of a
    32-point unit's rows): a channel overflows when a lane's K-th kept value is
    still inside the band (a dropped point might be the argmax)."""
    p = make_params(cls_spec(40), 0)
    rng = np.random.default_rng(1000)
    N = 1024
    pts = rng.uniform(-1, 1, (clouds, N, 3)).astype(F32)
    _, _, x3 = point_mlp_fwd(pts, p)
    w32 = p["feat.conv4.weight"].reshape(1024, 128).astype(F32)
    w = w32.astype(np.float64)
    whi = bf16_round(w32).astype(np.float64)
    wlo = bf16_round((w32 - whi.astype(F32)).astype(F32)).astype(np.float64)
    wn = np.linalg.norm(w, axis=1)
    dwn = np.linalg.norm(w - whi, axis=1)
    half = (np.arange(N) % 32 >> 2) & 1
    out = [f"two-product screens over {clouds} clouds x 1024 channels (configs[2] inputs)"]
    for form in ("A: (x_hi + x_lo) . w_hi", "B: x_hi . (w_hi + w_lo)"):
        cand_pp, cand_u, ovf = [], [], {2: 0, 3: 0, 4: 0}
        errs = []
        for b in range(clouds):
            x32 = x3[b].astype(F32)
            x = x32.astype(np.float64)
            xhi = bf16_round(x32).astype(np.float64)
            xlo = bf16_round((x32 - xhi.astype(F32)).astype(F32)).astype(np.float64)
            xn = np.linalg.norm(x, axis=1)
            v = x @ w.T
            if form[0] == "A":
                s = (xhi + xlo) @ whi.T
                e = xn[:, None] * dwn[None, :]
            else:
                s = xhi @ (whi + wlo).T
                e = np.linalg.norm(x - xhi, axis=1)[:, None] * wn[None, :]
            e = e + 2.0 ** -15 * xn[:, None] * wn[None, :]
            errs.append((np.abs(v - s) / e).max())
            inb = s + e >= (s - e).max(0)[None, :]
            cand_pp.append(inb.sum(0))
            eu = e.max(0)
            inu = s >= (s.max(0) - 2 * eu)[None, :]
            cand_u.append(inu.sum(0))
            for K in ovf:
                # lane h's K-th largest kept value inside the uniform band
                ov = np.zeros(1024, bool)
                for h in (0, 1):
                    sh = np.where(half[:, None] == h, s, -np.inf)
                    kth = -np.sort(-sh, axis=0)[K - 1]
                    ov |= kth >= s.max(0) - 2 * eu
                ovf[K] += int(ov.sum())
        tot = clouds * 1024
        a, u = np.concatenate(cand_pp), np.concatenate(cand_u)
        out.append(f"{form}: max |v - s| / bound = {max(errs):.3f}")
        out.append(f"  candidates, per-point band:  mean {a.mean():.2f} p99 {np.percentile(a, 99):.0f} "
                   f"max {a.max()}")
        out.append(f"  candidates, uniform band:    mean {u.mean():.2f} p99 {np.percentile(u, 99):.0f} "
                   f"max {u.max()}")
        for K, n in ovf.items():
            out.append(f"  top-{K} per lane, uniform band: overflow on {n} / {tot} channels "
                       f"({100 * n / tot:.2f} %)")
    return "\n".join(out)


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    print(main(n))
    print(two_product(n))
