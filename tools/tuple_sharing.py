"""Would k_weak_cand_comb gain from computing the focal anchor term once per anchor tuple? (VERDICT r4
item 5.) ComputeBilateralNCCNew's strong_costs + Softmax (APD.cu:488-587) depend on the pixel only
through its ordered anchors[1..8], their SA-used bits, the candidate plane and the view; the centre
window and the out-of-frame rule of the centre are per pixel. For the bench's headline problem (or
W H N) after apd_stage_prepare this counts the distinct ordered anchor tuples (with their used bits:
all valid anchors without SA masks) among the WEAK pixels, and the distinct (tuple, candidate anchor)
keys, against the per-pixel work k_weak_cand_comb does today.
Usage (GPU box): python tools/tuple_sharing.py [W H N]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import bench  # noqa: E402
import apd_abi as A  # noqa: E402

W, H, N = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (6048, 4032, 10)
sc = bench.make_scene(W, H, N, 1, os.environ.get("AB_TEXTURE", "smooth"))
eng = A.Engine(0, A.load_library())
ids = [0] + [j for j, _ in sc.pairs[0]][:N]
priors = bench.first_init_priors(eng, sc, ids, N)
arr = bench.final_round_problem(sc, priors, 0, N)
eng.set_problem(arr)
eng.prepare()
out = eng.results(A.Outputs(W, H, N, max_weak=W * H))
nw = int(out.weak_count[0])
strong = arr.weak_info.reshape(-1) == A.STRONG
anc = out.anchors[:nw].astype(np.int64)  # [nw, 9, 2] (x, y), row-major WEAK order
ok = (anc[..., 0] >= 0) & (anc[..., 1] >= 0)
q = np.where(ok, anc[..., 1] * W + anc[..., 0], -1)[:, 1:]  # anchors 1..8 (-1: none)
cand = ok[:, 1:] & strong[np.maximum(q, 0)]
print(f"{nw} WEAK px ({nw / (W * H):.3f}); valid anchors per px {ok[:, 1:].sum(1).mean():.2f}; "
      f"candidates per px {cand.sum(1).mean():.2f}", flush=True)
tup = np.ascontiguousarray(q).view(np.dtype((np.void, 8 * 8))).ravel()
ut, inv, cnt = np.unique(tup, return_inverse=True, return_counts=True)
print(f"ordered anchor tuples: {ut.size} distinct -> sharing {nw / ut.size:.3f}x; pixels per tuple p50 "
      f"{np.percentile(cnt, 50):.0f} p90 {np.percentile(cnt, 90):.0f} p99 {np.percentile(cnt, 99):.0f} max {cnt.max()}; "
      f"pixels whose tuple is shared {float((cnt[inv] > 1).mean()):.3f}", flush=True)
# per (tuple, candidate anchor): the comb kernel's (pixel, candidate) items against the distinct ones
items = int(cand.sum())
keys = np.repeat(inv, 8)[cand.ravel()] * (W * H) + q.ravel()[cand.ravel()]
uk = np.unique(keys).size
print(f"(pixel, candidate) items {items}; distinct (tuple, candidate anchor) {uk} -> sharing {items / max(uk, 1):.3f}x",
      flush=True)
# unordered sets (an upper bound for any re-ordering scheme: the softmax sums in anchor order)
srt = np.sort(q, axis=1)
us = np.unique(np.ascontiguousarray(srt).view(np.dtype((np.void, 8 * 8))).ravel()).size
print(f"unordered anchor sets: {us} distinct -> sharing {nw / us:.3f}x (upper bound)", flush=True)
