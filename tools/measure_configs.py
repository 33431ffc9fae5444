"""Per-config measurements for BASELINE.md §5 (run on the GPU box from the repo root):
    python tools/measure_configs.py [C1 C2 C3 C4 ...] > out.json
For each config's synthetic stand-in it times, on one MI355X, a FIRST_INIT problem
and an APD + geometric-consistency REFINE_ITER problem (priors = FIRST_INIT outputs of the
neighbouring views, the data flow of main.cpp's rounds >= 1) for reference view 0:
  mpix_s_iter   W*H / median per-iteration device time (apd_get_timing.iter_ms, HIP events)
  mpix_s_e2e    W*H*max_iterations / RunPatchMatch device time (main.cpp:157-159 bracket)
C1 is the CPU oracle (BASELINE.md §5 row "C1 | CPU oracle"), timed with its own steady_clock hooks.
Accuracy vs the oracle is bit-exact by test (tests/test_gpu_parity.py, tests/test_gpu_fullsize.py),
so depth L1 = 0 and mask identity = 100 % wherever both run; GT accuracy is reported for the
synthetic scene."""
import json
import os
import statistics
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import apd_abi as A  # noqa: E402
import cases  # noqa: E402
import synth  # noqa: E402

CONFIGS = {
    "C1": dict(w=640, h=480, n=4, iters=2),
    "C2": dict(w=3024, h=2016, n=8),
    "C3": dict(w=6048, h=4032, n=10),
    "C4": dict(w=1920, h=1056, n=10, gf=0.05),
}


def gt_stats(out, gt):
    d = out.planes[..., 3]
    m = (gt > 0) & (out.weak_info != A.UNKNOWN)
    rel = np.abs(d[m] - gt[m]) / gt[m]
    return {"gt_median_rel_depth_err": round(float(np.median(rel)), 5),
            "gt_frac_within_1pct": round(float((rel < 0.01).mean()), 4), "valid_frac": round(float(m.mean()), 4)}


def time_problem(eng, arr, gt):
    eng.set_problem(arr)
    eng.run()
    t = eng.timing()
    out = eng.results(A.Outputs(arr.width, arr.height, len(arr.images) - 1, max_weak=arr.width * arr.height))
    iters = list(t.iter_ms)[: t.iterations]
    hw = arr.width * arr.height
    r = {"run_patchmatch_ms": round(t.total_ms, 1), "iter_ms": [round(x, 2) for x in iters],
         "prepare_ms": round(t.prepare_ms, 1), "init_ms_beside": round(t.init_ms, 1), "anchors_ms": round(t.anchors_ms, 1),
         "sweep_ms": round(t.sweep_ms, 1),
         "post_ms": round(t.post_ms, 1),
         "mpix_s_iter": round(hw / (statistics.median(iters) * 1e-3) / 1e6, 2) if iters else None,
         "mpix_s_e2e": round(hw * t.iterations / (t.total_ms * 1e-3) / 1e6, 2)}
    if arr.params.use_APD:
        r["weak_frac_in"] = round(float((arr.weak_info == A.WEAK).mean()), 4)
    r.update(gt_stats(out, gt))
    return r, out


def measure_gpu(name, cfg, eng):
    t0 = time.time()
    sc = synth.make_scene(cfg["w"], cfg["h"], cfg["n"], seed=20251114)
    res = {"config": name, "width": cfg["w"], "height": cfg["h"], "n_src": cfg["n"], "device": "1x MI355X",
           "scene_gen_s": round(time.time() - t0, 1)}
    gf = cfg.get("gf")

    def problem(r):
        arr = cases.base_problem(sc, r, cfg["n"])
        if gf is not None:
            arr.params.geom_factor = gf
        return arr

    first, _ = time_problem(eng, problem(0), sc.gt_depth[0])
    res["first_init"] = first
    priors = []
    for r in range(len(sc.images)):
        eng.set_problem(problem(r))
        eng.run()
        priors.append(eng.results(A.Outputs(cfg["w"], cfg["h"], cfg["n"])))
    arr = cases.refine_problem(sc, priors, 0, cfg["n"], state=A.REFINE_ITER, geom=True, apd=True)
    if gf is not None:
        arr.params.geom_factor = gf
    res["apd_geom_pass"], _ = time_problem(eng, arr, sc.gt_depth[0])
    return res


def measure_c1(cfg):
    import ctypes as C
    import oracle_lib
    sc = synth.make_scene(cfg["w"], cfg["h"], cfg["n"], seed=20251114)
    arr = cases.base_problem(sc, 0, cfg["n"])
    arr.params.max_iterations = cfg["iters"]
    lib = oracle_lib.load()
    threads = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    out = oracle_lib.run(lib, arr, threads)
    prep, sweep, post = out.times
    hw = cfg["w"] * cfg["h"]
    return {"config": "C1", "width": cfg["w"], "height": cfg["h"], "n_src": cfg["n"], "device": f"CPU oracle, {threads} threads",
            "max_iterations": cfg["iters"], "times_s": [round(x, 3) for x in out.times],
            "mpix_s_iter": round(hw * cfg["iters"] / sweep / 1e6, 4),
            "mpix_s_e2e": round(hw * cfg["iters"] / (prep + sweep + post) / 1e6, 4), **gt_stats(out, sc.gt_depth[0])}


def main():
    names = sys.argv[1:] or ["C1", "C2", "C3", "C4"]
    eng = None
    for name in names:
        cfg = CONFIGS[name]
        if name == "C1":
            r = measure_c1(cfg)
        else:
            eng = eng or A.Engine(0)
            r = measure_gpu(name, cfg, eng)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
