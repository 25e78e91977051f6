"""CPU model of the cached-neighbour test with a second chance inside the cached NN's kd leaf/subtree.

Diagnostic (float64 ICP on the benchmark pairs; not a parity tool).  For every ICP pass it counts the
queries the batched NN pass would have to search:
  base   the current test: d(X, t_j) < L - sum(delta) (L = second-nearest distance at the last search);
  blk    + on a miss, the targets of j's 16-point kd leaf are evaluated and the best one is exact when it
         is closer than Lo - |X - X_s|, Lo = nearest target outside that leaf at the search position X_s;
  sb     the same with j's 128-point subtree (superblock).
    python tools/experiments/second_chance_sim.py [pairs] [iters]
"""
from __future__ import annotations

import os
import sys

import numpy as np
from scipy.spatial import cKDTree

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "icp-4dradar_amd"))
from icp4r import synth  # noqa: E402


def kd_leaves(p, leaf=16):
    """Leaf id per point of a balanced kd order (median split of the widest axis, leaves of `leaf`)."""
    ids = np.empty(len(p), np.int64)
    stack = [(np.arange(len(p)), 0)]
    nxt = 0
    while stack:
        idx, _ = stack.pop()
        if len(idx) <= leaf:
            ids[idx] = nxt
            nxt += 1
            continue
        q = p[idx]
        ax = int(np.argmax(q.max(0) - q.min(0)))
        units = (len(idx) + leaf - 1) // leaf
        cut = (units // 2) * leaf
        o = idx[np.argsort(q[:, ax], kind="stable")]
        stack.append((o[cut:], 0))
        stack.append((o[:cut], 0))
    return ids


def umeyama(s, d):
    ms, md = s.mean(0), d.mean(0)
    H = (d - md).T @ (s - ms) / len(s)
    U, _, Vt = np.linalg.svd(H)
    S = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        S[2, 2] = -1
    R = U @ S @ Vt
    return R, md - R @ ms


def run(pair, iters):
    src = pair.src_xyzi()[:, :3].astype(np.float64)
    tgt = pair.tgt_xyzi()[:, :3].astype(np.float64)
    n = len(src)
    tree = cKDTree(tgt)
    blk = kd_leaves(tgt, 16)
    sb = blk // 8
    X = src.copy()
    st = None
    rows = []
    for it in range(iters + 1):
        d, j = tree.query(X, k=160)
        j1, d1, d2 = j[:, 0], d[:, 0], d[:, 1]
        lo_b = np.where(blk[j] != blk[j1][:, None], d, np.inf).min(1)
        lo_s = np.where(sb[j] != sb[j1][:, None], d, np.inf).min(1)
        if st is None:
            counts = (n, n, n)
            st = {m: dict(j=j1.copy(), L=d2.copy(), cum=np.zeros(n), Xs=X.copy(), lo=(lo_b if m == "blk" else lo_s).copy())
                  for m in ("base", "blk", "sb")}
        else:
            counts = []
            for m in ("base", "blk", "sb"):
                s = st[m]
                dj = np.linalg.norm(X - tgt[s["j"]], axis=1)
                hit = dj < s["L"] - s["cum"]
                assert (s["j"][hit] == j1[hit]).all()
                miss = ~hit
                if m != "base":
                    grp = blk if m == "blk" else sb
                    mv = np.linalg.norm(X - s["Xs"], axis=1)
                    # best target inside the cached NN's group; exact when closer than the group's bound
                    same = grp[j] == grp[s["j"]][:, None]
                    inside = np.where(same, d, np.inf)
                    best = inside.min(1)
                    sec = np.sort(inside, axis=1)[:, 1]
                    # groups larger than the 160 neighbours looked at: `inside` may miss members; only
                    # trust a hit whose best is the true NN (asserted) and whose bound excludes outside
                    ok = miss & (best < s["lo"] - mv)
                    assert (j[ok, np.argmin(inside[ok], axis=1)] == j1[ok]).all()
                    s["j"][ok] = j1[ok]
                    s["L"][ok] = np.minimum(sec[ok], s["lo"][ok] - mv[ok])
                    s["cum"][ok] = 0
                    miss &= ~ok
                counts.append(int(miss.sum()))
                s["j"][miss] = j1[miss]
                s["L"][miss] = d2[miss]
                s["cum"][miss] = 0
                s["Xs"][miss] = X[miss]
                s["lo"][miss] = (lo_b if m == "blk" else lo_s)[miss]
        rows.append(counts)
        if it == iters:
            break
        R, t = umeyama(X, tgt[j1])
        Xn = X @ R.T + t
        step = np.linalg.norm(Xn - X, axis=1)
        for s in st.values():
            s["cum"] += step
        X = Xn
    return np.array(rows)


def main():
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    tot = None
    for i in range(pairs):
        r = run(synth.make_pair(i, 8192), iters)
        tot = r if tot is None else tot + r
    q = pairs * 8192
    print("pass   base     blk      sb   (searched fraction)")
    for k, (a, b, c) in enumerate(tot):
        print(f"{k:4d} {a / q:7.3f} {b / q:7.3f} {c / q:7.3f}")
    s = tot[1:].sum(0) / (q * iters)
    print(f"passes 1..{iters}: base {s[0]:.3f}  blk {s[1]:.3f}  sb {s[2]:.3f}")


if __name__ == "__main__":
    main()
