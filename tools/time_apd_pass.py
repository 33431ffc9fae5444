"""Time one APD pass (REFINE_INIT + use_APD + geom) at bench size, priors from FIRST_INIT runs of the
neighbouring views (the data flow of main.cpp's round 1). Prints apd_get_timing and kernel shares."""
import os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import apd_abi as A, synth, cases
W, H, N = int(os.environ.get("AB_W", 3024)), int(os.environ.get("AB_H", 2016)), int(os.environ.get("AB_N", 8))
sc = synth.make_scene(W, H, N)
e = A.Engine(0)
def run(arr):
    e.set_problem(arr); e.run()
    return e.results(A.Outputs(arr.width, arr.height, len(arr.images) - 1))
t0 = time.time()
priors = [run(cases.base_problem(sc, r, N)) for r in range(len(sc.images))]
print(f"first pass over {len(sc.images)} views: {time.time() - t0:.1f}s", flush=True)
for state, geom in ((A.REFINE_INIT, False), (A.REFINE_ITER, True)):
    arr = cases.refine_problem(sc, priors, 0, N, state=state, geom=geom, apd=True)
    for rep in range(2):
        out = run(arr)
        t = e.timing()
        wc = int(np.sum(arr.weak_info == A.WEAK))
        print(f"state={state} geom={geom}: total {t.total_ms:.1f} ms anchors {t.anchors_ms:.1f} init {t.init_ms:.1f} "
              f"sweep {t.sweep_ms:.1f} post {t.post_ms:.1f} iters {[round(x, 1) for x in list(t.iter_ms)[:3]]} "
              f"weak px {wc} ({100 * wc / (W * H):.0f}%)", flush=True)
