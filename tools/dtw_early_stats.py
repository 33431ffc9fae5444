"""How many of DepthToWeak's pixels the inner disparity band decides (APD.cu:2200-2248): a pixel whose
curve has no local minimum i with |i - 30| <= weak_peak_radius and cost <= 0.5 is WEAK whatever its
other disparities give (the global minimum peak is then outside the radius or above 0.5, or there is
no peak). Runs the bench's headline pass (and a FIRST_INIT problem) at C3 with the curves exported and
prints the decided fraction of the active pixels. Usage (GPU box): python tools/dtw_early_stats.py"""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import bench
import apd_abi as A
import cases

W, H, N = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (6048, 4032, 10)
sc = bench.make_scene(W, H, N, 1, os.environ.get("AB_TEXTURE", "smooth"))
eng = A.Engine(0, A.load_library())
ids = [0] + [j for j, _ in sc.pairs[0]][:N]
priors = bench.first_init_priors(eng, sc, ids, N)


def stats(arr, label):
    arr.params.export_reliable_curve = 1
    R = int(arr.params.weak_peak_radius)
    eng.set_problem(arr)
    eng.run()
    out = eng.results(A.Outputs(W, H, N, want_curve=True))
    pc = out.reliable_curve  # [HW, 61]
    act = np.any(pc != 0.0, axis=1)
    c = pc[act]
    i = np.arange(2, 59)
    peak = (c[:, i - 1] > c[:, i]) & (c[:, i + 1] > c[:, i])
    inner = (np.abs(i - 30) <= R)[None, :] & (c[:, i] <= 0.5)
    keep = np.any(peak & inner, axis=1)
    state = np.asarray(out.weak_info).reshape(-1)[act] if hasattr(out, "weak_info") else None
    print(f"{label}: R={R} active {act.sum()} of {W * H}; decided WEAK by the inner band {1 - keep.mean():.4f}"
          + (f"; WEAK overall {(state == A.WEAK).mean():.4f}" if state is not None else ""), flush=True)
    if state is not None:  # (the output states pass later filters; printed as a cross-check only)
        print(f"  of the decided pixels WEAK in the output: {(state[~keep] == A.WEAK).mean():.4f}", flush=True)


stats(cases.base_problem(sc, 0, N), "FIRST_INIT")
stats(bench.final_round_problem(sc, priors, 0, N), "headline pass (REFINE_ITER + APD + geom, final round)")
