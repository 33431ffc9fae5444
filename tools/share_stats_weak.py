"""Tap sharing available to the Weak-candidate kernel's centre windows (CPU study).

k_weak_cand_vm evaluates, per WEAK pixel p, view and candidate (STRONG anchor q's plane), the 6x6
centre window around p under q's plane. The homography depends only on (plane, view), so pixels of
one group that evaluate the same anchor plane and share the window-grid parity (px & 1, py & 1) sample
identical taps where their windows overlap. This runs an oracle APD pass on a synthetic view,
groups the WEAK pixels into 8x8 blocks and reports centre-window taps against distinct samples.

    python tools/share_stats_weak.py [W H N]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]

import apd_abi as A  # noqa: E402
import cases  # noqa: E402
import oracle_lib  # noqa: E402


def main():
    W, H, N = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (252, 168, 4)
    lib = oracle_lib.load()
    sc = cases.scene(W, H, N)
    priors = cases.first_pass(lambda arr: oracle_lib.run(lib, arr), sc, N)
    arr = cases.refine_problem(sc, priors, 0, N, state=A.REFINE_ITER, geom=True, apd=True)
    weak_in = arr.weak_info.copy()
    out = oracle_lib.run(lib, arr)
    wk = out.weak_count[0]
    anchors = out.anchors[:wk]
    ys, xs = np.nonzero(weak_in == A.WEAK)  # raster order = the WEAK index order (anchors_map)
    tot = uni = 0
    groups = {}
    for idx, (py, px) in enumerate(zip(ys.tolist(), xs.tolist())):
        if idx >= wk:
            break
        g = (py // 8, px // 8)
        for k in range(1, 9):
            ax, ay = int(anchors[idx, k, 0]), int(anchors[idx, k, 1])
            if ax < 0 or ay < 0 or weak_in[ay, ax] != A.STRONG:
                continue
            groups.setdefault(g, {}).setdefault((ay, ax, py & 1, px & 1), []).append((py, px))
    for keys in groups.values():
        for users in keys.values():
            tot += 36 * len(users)
            pos = {(py - 5 + 2 * j, px - 5 + 2 * i) for py, px in users for i in range(6) for j in range(6)}
            uni += len(pos)
    print(f"{W}x{H} N={N}: WEAK {wk}, groups {len(groups)}, centre-window taps {tot}, distinct samples {uni}"
          f" (x{tot / max(uni, 1):.2f})")


if __name__ == "__main__":
    main()
