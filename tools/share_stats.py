"""How many window taps of the Strong sweep's propagated hypotheses could be shared (CPU study).

The homography of a plane depends only on the plane and the source view (APD.cu:334-394), so the
bilinear sample at reference position (x, y) under the plane of pixel q is the same value in every
window that evaluates q's plane. Same-colour pixels that pick the same neighbour q (adaptive
checkerboard, APD.cu:1119-1314) and share the lattice parity of their window grids (offsets
(+-1, +-3, +-5)) therefore share taps. This script runs the oracle on a synthetic view, replays the
neighbour choice of one launch on the final cost map, groups pixels into 64-pixel workgroup regions
(8 rows x 16 columns, one colour) and reports the taps per workgroup against the distinct
(q, lattice, position) samples (exact union and per-(q, lattice) bounding boxes).

    python tools/share_stats.py [W H N]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]

import cases  # noqa: E402
import oracle_lib  # noqa: E402


def picks(costs, colour):
    H, W = costs.shape
    out = []  # (py, px, qy, qx)
    ys, xs = np.nonzero(((np.arange(H)[:, None] + np.arange(W)[None, :]) & 1) == colour)
    for py, px in zip(ys.tolist(), xs.tolist()):
        def far(dy, dx, ok):
            best = None
            for i in range(11):
                y, x = py + dy * (3 + 2 * i), px + dx * (3 + 2 * i)
                if i == 0 and not ok(0):
                    return None
                if i > 0 and not ok(i):
                    continue
                if best is None or costs[y, x] < costs[best]:
                    best = (y, x)
            return best
        qs = []
        qs.append(far(-1, 0, lambda i: py > 2 + 2 * i))
        qs.append(far(1, 0, lambda i: py < H - 3 - 2 * i))
        qs.append(far(0, -1, lambda i: px > 2 + 2 * i))
        qs.append(far(0, 1, lambda i: px < W - 3 - 2 * i))

        def near(valid, start, cands):
            if not valid:
                return None
            best = start
            for ok, y, x in cands:
                if ok and costs[y, x] < costs[best]:
                    best = (y, x)
            return best
        qs.append(near(py > 0, (py - 1, px), [c for i in range(3) for c in (
            (py > 1 + i and px > i, py - 2 - i, px - 1 - i), (py > 1 + i and px < W - 1 - i, py - 2 - i, px + 1 + i))]))
        qs.append(near(py < H - 1, (py + 1, px), [c for i in range(3) for c in (
            (py < H - 2 - i and px > i, py + 2 + i, px - 1 - i), (py < H - 2 - i and px < W - 1 - i, py + 2 + i, px + 1 + i))]))
        qs.append(near(px > 0, (py, px - 1), [c for i in range(3) for c in (
            (px > 1 + i and py > i, py - 1 - i, px - 2 - i), (px > 1 + i and py < H - 1 - i, py + 1 + i, px - 2 - i))]))
        qs.append(near(px < W - 1, (py, px + 1), [c for i in range(3) for c in (
            (px < W - 2 - i and py > i, py - 1 - i, px + 2 + i), (px < W - 2 - i and py < H - 1 - i, py + 1 + i, px + 2 + i))]))
        for q in qs:
            if q is not None:
                out.append((py, px, q[0], q[1]))
    return np.array(out, np.int64)


def main():
    W, H, N = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (376, 252, 8)
    sc = cases.scene(W, H, N)
    arr = cases.base_problem(sc, 0)
    out = oracle_lib.run(oracle_lib.load(), arr)
    costs = out.costs
    P = picks(costs, 0)
    wg = (P[:, 0] // 8) * ((W + 15) // 16) + P[:, 1] // 16
    tot = box = uni = 0
    nkeys = []
    for g in np.unique(wg):
        S = P[wg == g]
        tot += 36 * len(S)
        keys = {}
        for py, px, qy, qx in S.tolist():
            keys.setdefault((qy, qx, py & 1, px & 1), []).append((py, px))
        nkeys.append(len(keys))
        for users in keys.values():
            u = np.array(users)
            box += ((u[:, 0].max() - u[:, 0].min()) // 2 + 6) * ((u[:, 1].max() - u[:, 1].min()) // 2 + 6)
            pos = set()
            for py, px in users:
                for i in range(6):
                    for j in range(6):
                        pos.add((py - 5 + 2 * j, px - 5 + 2 * i))
            uni += len(pos)
    print(f"{W}x{H} N={N}: picks {len(P)}, workgroups {len(np.unique(wg))}, keys/wg {np.mean(nkeys):.1f}")
    print(f"taps {tot}, union {uni} (x{tot / uni:.2f}), boxes {box} (x{tot / box:.2f})")


if __name__ == "__main__":
    main()
