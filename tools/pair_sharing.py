"""How often the Weak-candidate kernel's anchor windows repeat beyond one 64-pixel group: for the
bench's headline problem (or W H N) after apd_stage_prepare, counts the (window anchor, candidate
anchor) pairs ComputeBilateralNCCNew evaluates for the anchor candidates (APD.cu:500-575) and the
distinct ones within groups of 64, 256, 1024, 4096 WEAK pixels (8x8-tile order) and within a band
of rows. SA masks are ignored (the headline has none).
Usage: python tools/pair_sharing.py [W H N]"""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import bench
import apd_abi as A

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
weak = arr.weak_info.reshape(-1) == A.WEAK
strong = arr.weak_info.reshape(-1) == A.STRONG
wpix = np.flatnonzero(weak)[:nw]  # anchors are indexed by the raster rank of the WEAK pixel
anc = out.anchors[:nw].astype(np.int64)
ok = (anc[..., 0] >= 0) & (anc[..., 1] >= 0)
q = np.where(ok, anc[..., 1] * W + anc[..., 0], -1)
win = ok[:, 1:]
cand = win & strong[np.maximum(q[:, 1:], 0)]
# 8x8-tile order of the WEAK pixels
y, x = wpix // W, wpix % W
order = np.lexsort((x % 8 + 8 * (y % 8), x // 8, y // 8))
print(f"{nw} WEAK px; windows per px {win.sum(1).mean():.2f}; candidates per px {cand.sum(1).mean():.2f}", flush=True)


def pairs_of(sel):
    """(window anchor, candidate anchor) keys of the WEAK pixels `sel` (indices into the WEAK list)."""
    qs = q[sel, 1:]
    w, c = win[sel], cand[sel]
    keys = qs[:, :, None] * (W * H) + qs[:, None, :]  # [px, k, h]
    m = w[:, :, None] & c[:, None, :]
    return keys[m]


total = 0
band_rows = int(os.environ.get("BAND_ROWS", 256))
for g in (64, 256, 1024, 4096):
    tot, dist = 0, 0
    n = (nw // g) * g
    step = max(1, (n // g) // 2000)  # sample up to ~2000 groups
    for s in range(0, n, g * step):
        k = pairs_of(order[s:s + g])
        tot += k.size
        dist += np.unique(k).size
    print(f"groups of {g:5d}: evaluations {tot}, distinct {dist}, sharing {tot / max(dist, 1):.2f}x", flush=True)
for y0 in (H // 4, H // 2):
    sel = np.flatnonzero((y >= y0) & (y < y0 + band_rows))
    k = pairs_of(sel)
    print(f"band rows {y0}..{y0 + band_rows} ({sel.size} px): evaluations {k.size}, distinct {np.unique(k).size}, "
          f"sharing {k.size / max(np.unique(k).size, 1):.2f}x", flush=True)
if os.environ.get("GLOBAL") == "1":  # the whole image (sorts ~1.4 G keys: minutes)
    k = np.unique(pairs_of(np.arange(nw)))
    qk = k // (W * H)
    _, cnt = np.unique(qk, return_counts=True)
    tot = int(win.sum(1) @ np.ones(1) * 0) if False else int((win[:, :, None] & cand[:, None, :]).sum())
    print(f"whole image: evaluations {tot}, distinct {k.size}, sharing {tot / max(k.size, 1):.2f}x; "
          f"{cnt.size} distinct window anchors, candidates per window anchor mean {cnt.mean():.1f} "
          f"p50 {np.percentile(cnt, 50):.0f} p99 {np.percentile(cnt, 99):.0f} max {cnt.max()}", flush=True)
    ca = np.unique(q[:, 1:][cand])
    print(f"distinct candidate anchors {ca.size}", flush=True)
