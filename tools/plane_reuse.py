"""How many Weak-candidate costs could be carried over between iterations: runs the bench's headline
problem (or W H N) iteration by iteration through the staged entry points and reports, per
iteration i >= 1, the fraction of STRONG pixels whose plane is bit-identical to iteration i-1's and
the fraction of (WEAK pixel, candidate) pairs whose candidate plane (its STRONG anchor's) is.
Usage: python tools/plane_reuse.py [W H N]"""
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
strong = arr.weak_info == A.STRONG
eng.set_problem(arr)
eng.prepare()
prev = None
for i in range(arr.params.max_iterations):
    eng.iteration(i)
    eng.synchronize()
    out = eng.results(A.Outputs(W, H, N, max_weak=W * H))
    planes = out.planes.view(np.uint32).reshape(H, W, 4)
    if prev is not None:
        same = np.all(planes == prev, axis=2)
        nw = int(out.weak_count[0])
        anc = out.anchors[:nw, 1:, :].astype(np.int64)  # anchors 1..8 of each WEAK pixel
        ok = (anc[..., 0] >= 0) & (anc[..., 1] >= 0)
        q = np.where(ok, anc[..., 1] * W + anc[..., 0], 0)
        cand = ok & strong.reshape(-1)[q]
        cs = same.reshape(-1)[q] & cand
        print(f"iteration {i}: STRONG planes unchanged {same[strong].mean():.4f} "
              f"({int(strong.sum())} STRONG px); candidates unchanged {cs.sum() / max(cand.sum(), 1):.4f} "
              f"({int(cand.sum())} candidates over {nw} WEAK px); distinct anchors unchanged "
              f"{np.unique(q[cs]).size}/{np.unique(q[cand]).size}", flush=True)
    prev = planes.copy()
