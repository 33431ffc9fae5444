"""Tap sharing of the Weak candidates' centre windows at C3 (k_weak_cand_g's work): per group of G
consecutive WEAK pixels of the candidate list (16x... tile order, as k_weak_cand_g's workgroups), the
centre-window taps (6x6, step 2, around anchor 0) of every (pixel, candidate anchor q) pair are keyed
by (q, x, y): a sample at (x, y) under q's plane is the same value for every pixel of the group that has
q as a candidate. Prints total taps / distinct keys (the reduction a per-group sample table could
reach) for sampled groups. Usage (GPU box): python tools/centre_sharing.py [groups] [G]"""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import bench
import apd_abi as A

NG = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
G = int(sys.argv[2]) if len(sys.argv) > 2 else 64
W, H, N = 6048, 4032, 10
sc = bench.make_scene(W, H, N, 1, os.environ.get("AB_TEXTURE", "smooth"))
eng = A.Engine(0)
ids = [0] + [j for j, _ in sc.pairs[0]][:N]
priors = bench.first_init_priors(eng, sc, ids, N)
arr = bench.final_round_problem(sc, priors, 0, N)
eng.set_problem(arr)
eng.prepare()
weak = np.asarray(arr.weak_info)
nw = int((weak == A.WEAK).sum())
out = A.Outputs.__new__(A.Outputs)
anchors = np.zeros((nw, 9, 2), np.int16)
wc = np.zeros(1, np.int32)
s = A.ApdOutputs()
s.anchors = A._ptr(anchors, A.C.c_int16)
s.weak_count = A._ptr(wc, A.C.c_int32)
eng._check(eng.lib.apd_get_results(eng.ctx, A.C.byref(s)), "apd_get_results")
assert int(wc[0]) == nw
# WEAK index = raster rank; the candidate list = WEAK pixels in list-tile order (tile 8 x 32, 4x4 micro-tiles)
tw, th = 8, 32
ys, xs = np.nonzero(weak == A.WEAK)
wi_of = np.full(weak.shape, -1, np.int64)
wi_of[ys, xs] = np.arange(nw)
tiles_x = (W + tw - 1) // tw
tile = (ys // th) * tiles_x + (xs // tw)
lx, ly = xs % tw, ys % th
micro = (ly // 4) * (tw // 4) + (lx // 4)
k = micro * 16 + (ly % 4) * 4 + (lx % 4)
order = np.lexsort((k, tile))
wl = wi_of[ys[order], xs[order]]
rng = np.random.default_rng(1)
starts = rng.choice(max(1, nw // G), size=min(NG, max(1, nw // G)), replace=False) * G
di, dj = np.meshgrid(np.arange(6) * 2 - 5, np.arange(6) * 2 - 5, indexing="ij")
di, dj = di.ravel(), dj.ravel()
tot = dist = 0
for st in starts:
    g = wl[st:st + G]
    a = anchors[g].astype(np.int64)              # [G, 9, 2]
    a0 = a[:, 0]
    cand = a[:, 1:]                               # [G, 8, 2]
    ok = (cand[..., 0] >= 0) & (cand[..., 1] >= 0) & (a0[:, None, 0] >= 0)
    cx, cy = np.clip(cand[..., 0], 0, W - 1), np.clip(cand[..., 1], 0, H - 1)
    ok &= weak[cy, cx] == A.STRONG
    q = cy * W + cx                               # candidate anchor position
    px = a0[:, None, None, 0] + di[None, None, :]  # [G, 1, 36]
    py = a0[:, None, None, 1] + dj[None, None, :]
    key = (q[:, :, None] * 65536 + (px + 16)) * 65536 + (py + 16)
    key = key[np.broadcast_to(ok[:, :, None], key.shape)]
    tot += key.size
    dist += np.unique(key).size
print(f"C3 {os.environ.get('AB_TEXTURE', 'smooth')}: {len(starts)} groups of {G} WEAK pixels: centre-window taps {tot}, "
      f"distinct (candidate anchor, x, y) samples {dist}, sharing {tot / max(dist, 1):.2f}x", flush=True)
