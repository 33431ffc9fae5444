"""Benchmark: Mpix/s per PatchMatch iteration on the north-star workload, BASELINE.json configs[2].

Workload ("C3"): a synthetic ETH3D-office-shaped scan at full resolution,
6048x4032, one reference view + 10 source views, the final round's geometric pass of main.cpp
(main.cpp:333-365 with i = 3: REFINE_ITER, deformable PatchMatch (APD) with focal-weighted anchors,
geometric consistency, impetus, rotate_time 4, ransac_threshold 0.00625). Its priors (depths,
normals, pixel states, confidence of every view) come from FIRST_INIT runs of the scan's views at the
same resolution. A "step" is one iteration of the loop body APD.cu:2699-2708 over the whole
reference view: Strong sweep black + red, RANSACToGetFitPlane, and the Weak sweep black + red
(anchor candidates through the image-wide pair table: k_gp_cost + k_weak_cand_g + k_weak_cand_comb, then
k_sweep_weak_vm). Steps are iterations 0, 1, 2 of FRESH runs (the
median over a fresh run's iterations): before every block of (up to) 3 steps the problem is
re-uploaded and re-initialised (apd_set_problem + apd_stage_prepare, outside the timed region), so
no step repeats an iteration on an already-converged view. Each block is bracketed by a barrier and
a device synchronisation, and the blocks' times are summed; inputs are resident in HBM throughout.
The per-pass image-wide pair table (built in apd_stage_prepare; it replaces candidate work the
reference does inside every CheckerboardPropagationWeak, APD.cu:1442-1615) is charged to the steps:
each block adds its own build's HIP-event time x (its steps / 3).
value = W*H*steps summed over ranks / max-over-ranks (timed steps + charged pair tables);
mpix_s_iter_loop is the same without the pair tables (the loop body alone).

Multi-GPU (weak scaling): one process per GPU. `python3 bench.py --gpus N` outside a
torch.distributed launch starts its N ranks itself (a torch.distributed.run child on 127.0.0.1,
before anything in this process touches the GPU) and exits with the child's status; under the
driver's own torch.distributed.run it runs as one rank. Each rank runs its own reference view
(rank mod #views) of the same final-round pass with its own priors. Within a pass the reference
views are independent given the previous pass's view states (APD.cpp:592-610), and
the scan runner (apde-mvs_amd/scan_runner.py) ends every pass with ONE all-gather of the
new states (18 B/px on the wire: depth + normal xyz f32, pixel state + confidence u8). The bench does
the same inside the timed region: a scan pass gives every rank ceil(scan_views / N) problems, so after
that many blocks of fresh iterations (and after the last block) the ranks all-gather the states they
produced over RCCL (xGMI), and `value` at N > 1 pays the exchange; `exchange_ms` is the median of
separately timed all-gathers (barrier, then the collective alone) and `rank_ms_per_step` the ranks'
own per-step times (the value uses the max over ranks).

Besides the headline the JSON line carries:
  roofline      the dominant kernels of the step, the Weak sweep (the anchor candidates -- k_gp_cost +
                k_weak_cand_g + k_weak_cand_comb -- + 2 x k_sweep_weak_vm,
                95 % of it at C3): algorithmic FP32 flops = NCC-New evaluations x 4038 +
                geometric terms x 80, both counted on the device for the evaluations
                CheckerboardPropagationWeak uses (apd_profile_counters), / their summed launch time from
                HIP events on the engine stream, against the FP32 vector peak; HBM bytes per launch from
                the rocprofv3 PMC summary of k_sweep_weak_vm at this shape under profiles/ whose
                source_hash matches this tree's kernel sources (else traffic is null).
  cpu_baseline  the C oracle (oracle/liboracle.so) on a bounded sample of the same workload: the
                same scene rendered at W/4 x H/4 (1512x1008) with its textures scaled 4x in world
                units (the headline's texture per pixel and WEAK fraction), N = 10, one APD iteration
                of the same pass, at --cpu-threads cores; plus the same at 1 core on W/16 x H/16
                (378x252, textures scaled 16x: cpu_baseline_1core).
  end_to_end    one full RunPatchMatch of the headline problem (main.cpp:157-161 bracket).
  c2_first_init configs[1] (3024x2016, N = 8, FIRST_INIT, Strong sweep only): the round-1/2 headline,
                same fresh-run timing, with the Strong sweep's NCC-Old roofline.
  rich_texture  the headline pass on the texture-rich variant of the scene (synth texture="rich":
                fine detail + more textureless patches, WEAK fraction 30-50 % instead of ~94 %).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import statistics
import sys
import time
from types import SimpleNamespace

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402

METRIC = "Mpix/s per PatchMatch iteration (ref view, N src) at 1/2/4/8 GPU; depth L1 vs ref"
FLOP_PER_NCC_OLD = 36 * 36 + 150   # 36 samples x 36 flop + homography/finalise
FLOP_PER_NCC_NEW = 108 * 36 + 150  # <= 108 samples (6x6 centre + 8 anchors x 3x3)
FLOP_PER_GEOM = 80                 # one geometric-consistency term
FLOP_PER_TAP = 36                  # one bilinear NCC sample (projection, lerp, moments)
PEAK_FP32_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector peak (packed FP32)
PEAK_HBM_GBS = 8000.0
FINAL_ROUND = 3  # C3 has 4 rounds (6048 -> 756 halvings, main.cpp:129-146); the headline is round 3


def workload_name(W, H, N, apd):
    known = {(6048, 4032, 10, True): "C3", (3024, 2016, 8, False): "C2"}
    return known.get((W, H, N, apd), "custom")


KERNEL_SOURCES = ("apde-mvs_amd/csrc/apd_kernels.hip", "apde-mvs_amd/csrc/apd_device.h")


def source_hash() -> str:
    """sha256 (first 16 hex digits) of the kernel sources libapd_hip.so is built from: a PMC summary
    carries the hash of the sources it was collected with (tools/pmc_c3.sh), and only a summary whose
    hash matches the tree's is taken as this build's traffic."""
    import hashlib
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        with open(os.path.join(REPO, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def latest_pmc(kernel: str, W: int, n_src: int):
    """The PMC summary under profiles/ for this kernel and shape collected from THIS build's kernel
    sources (its source_hash equals source_hash()), or None: a summary of another build (a superseded
    variant, an older round) is never reported as the current traffic. Among matching files the
    newest by name wins. Counter studies of other shapes are skipped."""
    want = source_hash()
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc*.json")), reverse=True):
        try:
            pmc = json.load(open(f))
        except Exception:
            continue
        if (isinstance(pmc, dict) and str(pmc.get("kernel", "")).startswith(kernel)
                and pmc.get("width") == W and pmc.get("n_src") == n_src
                and pmc.get("hbm_bytes_per_launch") is not None and pmc.get("source_hash") == want):
            pmc["_file"] = os.path.relpath(f, REPO)
            return pmc
    return None


def fetch_calibration():
    """The measured FETCH_SIZE correction for this repo's gather widths (tools/fetch_calib.hip): HBM bytes
    = factor x FETCH_SIZE + WRITE_SIZE, the factor the PMC summaries' hbm_bytes_per_launch applies."""
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*fetch_calibration*.json")), reverse=True):
        try:
            c = json.load(open(f))
        except Exception:
            continue
        c["_file"] = os.path.relpath(f, REPO)
        return c
    return None


def make_scene(W, H, N, world, texture, texture_scale=1.0):
    import synth
    return synth.make_scene(W, H, max(N, world), seed=20251114, texture=texture, texture_scale=texture_scale)


def first_init_priors(eng, sc, ids, N):
    """FIRST_INIT runs (round 0's data flow) of the views in `ids`: per view the planes, pixel states
    and confidence the next pass reads as priors (main.cpp:306-331)."""
    import apd_abi as A
    W, H = sc.width, sc.height
    priors = {}
    for r in ids:
        arr = A.scene_problem(sc, r, [j for j, _ in sc.pairs[r]][:N], seed=0x5EED ^ r)
        eng.set_problem(arr)
        eng.run()
        out = SimpleNamespace(planes=np.zeros((H, W, 4), np.float32), weak_info=np.zeros((H, W), np.uint8),
                              confidence=np.zeros((H, W), np.uint8))
        s = A.ApdOutputs()
        s.planes = A._ptr(out.planes, A.C.c_float)
        s.weak_info = A._ptr(out.weak_info, A.C.c_uint8)
        s.confidence = A._ptr(out.confidence, A.C.c_uint8)
        eng._check(eng.lib.apd_get_results(eng.ctx, A.C.byref(s)), "apd_get_results")
        priors[r] = out
    return priors


def final_round_problem(sc, priors, ref, N, sa=False):
    """The REFINE_ITER + APD + geometric pass of main.cpp's last round (main.cpp:336-352, i = 3, j = 0);
    sa: with the reference view's SAM-style segment labels as the SA mask (config C5, APD.cpp:641-652)."""
    import apd_abi as A
    import cases
    arr = cases.refine_problem(sc, priors, ref, N, state=A.REFINE_ITER, geom=True, apd=True, sa=sa)
    arr.params.rotate_time = min(2 ** FINAL_ROUND, 4)
    arr.params.ransac_threshold = 0.01 - FINAL_ROUND * 0.00125
    arr.params.weak_peak_radius = max(4 - 2 * 0, 2)
    arr.params.use_impetus = 1
    return arr


PREP_LOG = []  # the timed blocks' prepare-phase timings (apd_get_prepare_timing), reported in the line


def timed_fresh_iterations(eng, arr, steps, warmup, barrier, exchange=None, exchange_every=1):
    """Warm-up, then `steps` loop-body iterations taken in blocks of one fresh run's iterations
    0..max_iterations-1; each block re-uploads and re-initialises the problem untimed, and is timed
    between a barrier + device synchronisation on both sides. `exchange(k)` (N > 1): the pass's
    all-gather of the k view states a rank produced since the last one, run inside the timed region
    after every `exchange_every` blocks (a scan pass: ceil(views / ranks) problems per rank, then one
    all-gather, scan_runner.py) and after the last block.
    The per-pass pair table (built in apd_stage_prepare: it replaces candidate work the reference
    does inside every CheckerboardPropagationWeak, APD.cu:1442-1615) is charged to the iterations:
    each block adds its own build's device time (apd_get_prepare_timing().pairs_ms, HIP events)
    times n / max_iterations for the n iterations it times.
    Returns (summed seconds incl. the charged pair tables, per-step ms, charged pair-table ms)."""
    iters = max(1, arr.params.max_iterations)
    done = 0
    while done < warmup:
        eng.set_problem(arr)
        eng.prepare()
        n = min(iters, warmup - done)
        for i in range(n):
            eng.iteration(i)
        done += n
    eng.synchronize()
    eng.profile_reset(True)
    elapsed, step_ms, done, pairs_ms, pending = 0.0, [], 0, 0.0, 0
    PREP_LOG.clear()
    while done < steps:
        eng.set_problem(arr)
        eng.prepare()
        eng.synchronize()
        pt = eng.prepare_timing()
        PREP_LOG.append({"pairs_ms": round(pt.pairs_ms, 2), "lists_ms": round(pt.lists_ms, 2), "init_ms": round(pt.init_ms, 2),
                         "prepare_ms": round(pt.prepare_ms, 2)})
        pairs_ms += pt.pairs_ms * min(iters, steps - done) / iters
        barrier()
        t_block = time.perf_counter()
        t_prev = t_block
        n = min(iters, steps - done)
        for i in range(n):
            eng.iteration(i)
            eng.synchronize()  # per-step times for the median (a few us against >=25 ms steps)
            t = time.perf_counter()
            step_ms.append((t - t_prev) * 1e3)
            t_prev = t
        pending += 1
        if exchange is not None and (pending == exchange_every or done + n >= steps):
            exchange(pending)
            pending = 0
            t_prev = time.perf_counter()
        elapsed += t_prev - t_block
        barrier()
        done += n
    return elapsed + pairs_ms * 1e-3, step_ms, pairs_ms


def kernel_stats(eng, kind):
    ms, n, px = eng.profile_kernel(kind)
    return {"ms_total": ms, "launches": n, "avg_ms": round(ms / n, 4) if n else None, "pixels": px}


def weak_roofline(eng, steps, W, N):
    """Roofline of the Weak sweep (candidate kernels + k_sweep_weak_vm) over the timed steps."""
    import apd_abi as A
    cnt = eng.profile_counters()
    cand = kernel_stats(eng, A.PROF_WEAK_CAND)
    sweep = kernel_stats(eng, A.PROF_WEAK_SWEEP)
    strong = kernel_stats(eng, A.PROF_STRONG_SWEEP)
    ransac = kernel_stats(eng, A.PROF_RANSAC_FIT)
    path = kernel_stats(eng, A.PROF_WEAK_PATH)
    # the Weak path's wall time: RANSACToGetFitPlane and k_gp_cost run on side streams beside
    # k_weak_cand_g, so the kernels' own brackets overlap; the path bracket (end of the Strong sweeps
    # to the end of the Weak sweeps, RANSAC included) is the time they take together
    ms = path["ms_total"] if path["launches"] else cand["ms_total"] + sweep["ms_total"]
    flop = cnt[1] * FLOP_PER_NCC_NEW + cnt[2] * FLOP_PER_GEOM
    achieved = flop / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
    # device-issued work: the windows the kernels actually evaluated (the pair table evaluates each
    # distinct (window anchor, candidate) window once per view; RandomInitialization's kept costs and
    # the exact early exit skip evaluations) -- 3x3 windows 9 taps, 6x6 centre windows 36 taps
    taps = 9 * (cnt[5] + cnt[8]) + 36 * (cnt[6] + cnt[7])
    flop_issued = taps * FLOP_PER_TAP + cnt[2] * FLOP_PER_GEOM
    achieved_issued = flop_issued / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
    pmc = latest_pmc("k_sweep_weak_vm", W, N)
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    cal = fetch_calibration()
    return {
        "bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
        "frac": round(achieved / PEAK_FP32_TFLOPS, 4), "traffic": traffic,
        "basis": "algorithmic (effective): the NCC-New evaluations CheckerboardPropagationWeak performs, "
                 "priced at SURVEY.md §8d's 4038 flop; achieved_issued / frac_issued price the windows the "
                 "kernels actually evaluated (36 flop per tap)",
        "achieved_issued": round(achieved_issued, 3), "frac_issued": round(achieved_issued / PEAK_FP32_TFLOPS, 4),
        "kernel": "k_sweep_weak_vm (+ k_gp_cost + k_weak_cand_g + k_weak_cand_comb): CheckerboardPropagationWeak, APD.cu:1442-1615",
        "note": "VALU-FP32 gather/stencil kernels (no matrix work, SURVEY.md §8d); one Weak sweep "
                "iteration = the anchor-candidate kernels (k_gp_cost + k_weak_cand_g + k_weak_cand_comb) + 2 k_sweep_weak_vm launches; flops = device-counted "
                "NCC-New x 4038 + geometric terms x 80, over the Weak path's HIP-event wall time (time_basis); "
                "traffic = HBM bytes per k_sweep_weak_vm launch (PMC, profiles/); launch_avg_ms are the kernels' "
                "own brackets (k_gp_cost and k_ransac_fit overlap k_weak_cand_g)",
        "ms_per_iteration": round(ms / max(steps, 1), 3),
        "time_basis": "wall time of the Weak path per iteration (end of the Strong sweeps to the end of the Weak sweeps, "
                      "RANSACToGetFitPlane running beside the candidate kernels included)" if path["launches"] else
                      "summed kernel brackets",
        "flop_per_iteration": flop / max(steps, 1),
        "ncc_new_per_iteration": round(cnt[1] / max(steps, 1)),
        "issued_windows_per_iteration": {"k_gp_cost 3x3": round(cnt[5] / max(steps, 1)),
                                         "k_weak_cand_g 6x6": round(cnt[6] / max(steps, 1)),
                                         "k_sweep_weak_vm 6x6": round(cnt[7] / max(steps, 1)),
                                         "k_sweep_weak_vm 3x3": round(cnt[8] / max(steps, 1))},
        "geom_terms_per_iteration": round(cnt[2] / max(steps, 1)),
        "launch_avg_ms": {"k_gp_cost+k_weak_cand_g+k_weak_cand_comb": cand["avg_ms"],
                          "k_gp_cost": kernel_stats(eng, A.PROF_GP_COST)["avg_ms"],
                          "k_weak_cand_g": kernel_stats(eng, A.PROF_WEAK_CAND_G)["avg_ms"],
                          "k_weak_cand_comb": kernel_stats(eng, A.PROF_WEAK_CAND_COMB)["avg_ms"],
                          "k_sweep_weak_vm": sweep["avg_ms"],
                          "k_sweep_strong_vm": strong["avg_ms"], "k_ransac_fit": ransac["avg_ms"]},
        "launches": {"k_gp_cost+k_weak_cand_g+k_weak_cand_comb": cand["launches"], "k_sweep_weak_vm": sweep["launches"],
                     "k_sweep_strong_vm": strong["launches"], "k_ransac_fit": ransac["launches"]},
        "pmc_file": pmc.get("_file") if pmc else None,
        "traffic_correction_factor": cal.get("correction_factor") if cal else None,
        "traffic_calibration": cal.get("_file") if cal else None,
    }


def strong_roofline(eng, W, N):
    """Roofline of the Strong sweep (k_sweep_strong_vm) over the profiled launches."""
    import apd_abi as A
    st = kernel_stats(eng, A.PROF_STRONG_SWEEP)
    evals = eng.profile_counters()[0]
    n = max(st["launches"], 1)
    launch_ms = st["ms_total"] / n
    flop = evals / n * FLOP_PER_NCC_OLD
    achieved = flop / (launch_ms * 1e-3) / 1e12 if launch_ms > 0 else 0.0
    pmc = latest_pmc("k_sweep_strong", W, N)
    return {"bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
            "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
            "kernel": "k_sweep_strong_vm: CheckerboardPropagationStrong, APD.cu:1098-1440",
            "launch_ms": round(launch_ms, 4), "launches": st["launches"], "flop_per_launch": flop,
            "ncc_evals_per_launch": round(evals / n)}


def gt_accuracy(sc, ref, eng, W, H, N):
    import apd_abi as A
    out = eng.results(A.Outputs(W, H, N))
    gt = sc.gt_depth[ref]
    d = out.planes[..., 3]
    m = (gt > 0) & (out.weak_info != A.UNKNOWN)
    rel = np.abs(d[m] - gt[m]) / gt[m]
    return {"gt_median_rel_depth_err": round(float(np.median(rel)), 5),
            "gt_frac_within_1pct": round(float((rel < 0.01).mean()), 4),
            "weak_frac_out": round(float((out.weak_info == A.WEAK).mean()), 4)}


def depth_to_weak_roofline(eng, W, N):
    """Roofline of DepthToWeak (k_depth_to_weak_vm, APD.cu:2103-2250) over the profiled launches:
    device-counted NCC-Old evaluations x 1446 + geometric terms x 80 / launch time."""
    import apd_abi as A
    st = kernel_stats(eng, A.PROF_DEPTH_TO_WEAK)
    cnt = eng.profile_counters()
    n = max(st["launches"], 1)
    launch_ms = st["ms_total"] / n
    flop = (cnt[3] * FLOP_PER_NCC_OLD + cnt[4] * FLOP_PER_GEOM) / n
    achieved = flop / (launch_ms * 1e-3) / 1e12 if launch_ms > 0 else 0.0
    pmc = latest_pmc("k_depth_to_weak_vm", W, N)
    return {"bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
            "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
            "pmc_file": pmc.get("_file") if pmc else None,
            "kernel": "k_depth_to_weak_vm: DepthToWeak, APD.cu:2103-2250",
            "launch_ms": round(launch_ms, 3), "launches": st["launches"], "flop_per_launch": flop,
            "ncc_old_per_launch": round(cnt[3] / n), "geom_terms_per_launch": round(cnt[4] / n)}


def end_to_end(eng, arr, sc, ref, W, H, N):
    """One full RunPatchMatch (the main.cpp:157-161 bracket), after an untimed one (first-use
    allocations and code loading out of the way). The timed run is unprofiled (only the phase events
    of apd_timing); a third, profiled run (HIP events around the loop-body kernels and DepthToWeak,
    device counters) gives DepthToWeak's roofline."""
    eng.set_problem(arr)
    eng.run()
    eng.set_problem(arr)
    eng.profile_reset(False)
    t1 = time.perf_counter()
    eng.run()
    t2 = time.perf_counter()
    tm = eng.timing()
    eng.set_problem(arr)
    eng.profile_reset(True)
    eng.run()
    dtw = depth_to_weak_roofline(eng, W, N)
    eng.profile_reset(False)
    iters = tm.iterations
    # RandomInitialization runs beside the lists and the pair table (side stream): the prepare phase
    # takes max(lists + pairs, init) of the ctx stream's time
    parts = tm.anchors_ms + max(tm.lists_ms + tm.pairs_ms, tm.init_ms) + tm.sweep_ms + tm.post_ms
    r = {"run_patchmatch_ms": round(tm.total_ms, 3), "host_wall_ms": round((t2 - t1) * 1e3, 3), "profiled": False,
         "mpix_s_end_to_end": round(W * H * iters / (tm.total_ms * 1e-3) / 1e6, 3),
         "anchors_ms": round(tm.anchors_ms, 3), "lists_ms": round(tm.lists_ms, 3), "pairs_ms": round(tm.pairs_ms, 3),
         "init_ms": round(tm.init_ms, 3), "sweep_ms": round(tm.sweep_ms, 3),
         "post_ms": round(tm.post_ms, 3), "accounted_frac": round(parts / tm.total_ms, 4) if tm.total_ms else None,
         "iter_ms": [round(x, 3) for x in list(tm.iter_ms)[:iters]], "roofline_depth_to_weak": dtw}
    r.update(gt_accuracy(sc, ref, eng, W, H, N))
    return r


def apd_pass_once(eng, sc, ref, N, label, sa=False):
    """Priors + one fresh timed pass (3 iterations) + end to end, for a secondary scene variant."""
    W, H = sc.width, sc.height
    ids = [ref] + [j for j, _ in sc.pairs[ref]][:N]
    priors = first_init_priors(eng, sc, ids, N)
    arr = final_round_problem(sc, priors, ref, N, sa=sa)
    el, step_ms, pairs = timed_fresh_iterations(eng, arr, arr.params.max_iterations, 1, lambda: None)
    roof = weak_roofline(eng, len(step_ms), W, N)
    eng.profile_reset(False)
    e2e = end_to_end(eng, arr, sc, ref, W, H, N)
    r = {"workload": label, "mpix_s_iter": round(W * H * len(step_ms) / el / 1e6, 3),
         "mpix_s_iter_loop": round(W * H * len(step_ms) / (el - pairs * 1e-3) / 1e6, 3),
         "pairs_ms_charged": round(pairs, 3),
         "iter_ms": [round(x, 2) for x in step_ms], "weak_frac": round(float((arr.weak_info == 0).mean()), 4),
         "roofline_frac": roof["frac"], "roofline_achieved": roof["achieved"],
         "launch_avg_ms": roof["launch_avg_ms"], "end_to_end": e2e}
    if sa:
        r["sa_labelled_frac"] = round(float((arr.sa_mask > 0).mean()), 4)
    return r


def c2_first_init(eng, steps, warmup):
    """configs[1]: 3024x2016, N = 8, FIRST_INIT (geom off, APD off): Strong sweep B + R per step."""
    import apd_abi as A
    W, H, N = 3024, 2016, 8
    sc = make_scene(W, H, N, 1, "smooth")
    arr = A.scene_problem(sc, 0, [j for j, _ in sc.pairs[0]][:N], seed=0x5EED)
    el, step_ms, _ = timed_fresh_iterations(eng, arr, steps, warmup, lambda: None)
    roof = strong_roofline(eng, W, N)
    eng.profile_reset(False)
    e2e = end_to_end(eng, arr, sc, 0, W, H, N)
    return {"workload": "C2: ETH3D-office-shaped scan, half-res 3024x2016, 1 ref + 8 src views, FIRST_INIT "
                        "(geom off, APD off), Strong sweep B + R per step, fresh runs",
            "value": round(W * H * len(step_ms) / el / 1e6, 3), "unit": "Mpix/s", "steps": len(step_ms),
            "ms_per_step": round(el / len(step_ms) * 1e3, 4),
            "iter_ms_median": round(statistics.median(step_ms), 3), "roofline": roof, "end_to_end": e2e}


def cpu_baseline(eng, texture, N, w, h, threads, W, H):
    """The C oracle on one APD iteration of the headline pass, on the same scene rendered at w x h
    with its smooth textures scaled by W / w in world units, so that the sample has the headline's
    texture per pixel and WEAK fraction (synth texture_scale); priors from FIRST_INIT runs on the
    device, which are bit-identical to the oracle's."""
    import ctypes as C
    import oracle_lib
    scale = W / w if texture == "smooth" else 1.0
    sc = make_scene(w, h, N, 1, texture, texture_scale=scale)
    ids = [0] + [j for j, _ in sc.pairs[0]][:N]
    priors = first_init_priors(eng, sc, ids, N)
    arr = final_round_problem(sc, priors, 0, N)
    lib = oracle_lib.load()
    pb = arr.build()
    times = (C.c_double * 3)()
    st = lib.oracle_time_iterations(C.byref(pb), 1, threads, times)
    if st != 0:
        return None
    t_iter = times[1]
    return {"value": round(w * h / t_iter / 1e6, 5), "unit": "Mpix/s", "cores": threads, "kind": "port",
            "weak_frac": round(float((arr.weak_info == 0).mean()), 4),
            "sample": f"oracle (C restatement{', OpenMP' if threads > 1 else ', 1 thread'}) on the headline "
                      f"pass (REFINE_ITER, APD + focal + geom + impetus, final-round params) of the same "
                      f"synthetic scan rendered at {w}x{h} with texture_scale {scale:g} (the headline's texture "
                      f"per pixel), N={N}, one loop-body iteration "
                      f"(t_iter={t_iter:.2f}s; anchors/RandomInit {times[0]:.2f}s untimed)"}


def self_launch_cmd(argv, gpus, env):
    """The torch.distributed.run command that starts `gpus` ranks of this script with the same
    arguments, or None when no launch is needed (one GPU, or already a rank of a distributed launch:
    WORLD_SIZE set by the driver's own torch.distributed.run). Built and run before anything in this
    process touches the GPU; the ranks rendezvous on 127.0.0.1 at a free port (APD_BENCH_PORT
    overrides it)."""
    if gpus <= 1 or "WORLD_SIZE" in env:
        return None
    port = env.get("APD_BENCH_PORT")
    if not port:
        import socket
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
            so.bind(("127.0.0.1", 0))
            port = str(so.getsockname()[1])
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def state_exchange(tdist, torch, state, world, kmax=1):
    """The scan runner's per-pass step (scan_runner.Exchange.all_gather_state): the k view
    states each rank produced to every rank, in the exchange's wire format (scan_runner.wire_pack:
    18 B/px, depth + normal f32, pixel state + confidence u8), device to device (RCCL over xGMI; gloo
    in the one-GPU rehearsal). Buffers for up to kmax states per rank are allocated here, outside the
    timed region. Returns (exchange, timed, wire_bytes): exchange(k) runs one all-gather of k states
    per rank and waits for it; timed(reps, k) is the median ms of `reps` all-gathers, each after a
    barrier (the collective alone, without the ranks' load imbalance)."""
    import scan_runner
    wire = scan_runner.wire_pack(state)
    buf = wire.unsqueeze(0).repeat(kmax, 1).contiguous()
    outs = [torch.empty_like(buf) for _ in range(world)]

    def exchange(k=1):
        tdist.all_gather([o[:k] for o in outs], buf[:k])
        if buf.is_cuda:
            torch.cuda.synchronize()

    def timed(reps, k=1):
        ms = []
        for _ in range(reps):
            tdist.barrier()
            if buf.is_cuda:
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            exchange(k)
            ms.append((time.perf_counter() - t0) * 1e3)
        return statistics.median(ms)
    return exchange, timed, int(wire.numel())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--width", type=int, default=6048)
    ap.add_argument("--height", type=int, default=4032)
    ap.add_argument("--n-src", type=int, default=10)
    ap.add_argument("--texture", default="smooth", choices=["smooth", "rich"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    ap.add_argument("--end-to-end", type=int, default=1, help="also time one full RunPatchMatch (0/1)")
    ap.add_argument("--c2", type=int, default=1, help="also measure configs[1] (C2 FIRST_INIT) (0/1)")
    ap.add_argument("--rich", type=int, default=1, help="also measure the texture-rich scene variant (0/1)")
    ap.add_argument("--sa", type=int, default=1, help="also measure the headline pass with SA labels (C5's pass) (0/1)")
    ap.add_argument("--scan-views", type=int, default=26,
                    help="views of the modelled scan (ETH3D office: 26): at N > 1 every rank runs "
                         "ceil(views / N) problems per pass, then the pass's all-gather")
    args = ap.parse_args()
    t_start_all = time.time()
    cmd = self_launch_cmd(sys.argv[1:], args.gpus, os.environ)
    if cmd is not None:
        # `python3 bench.py --gpus N`: start the N ranks as a child (nothing here has touched the GPU)
        import subprocess
        sys.exit(subprocess.call(cmd))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1 or args.gpus > 1:
        import torch
        import torch.distributed as tdist

        # nccl == RCCL on ROCm; APD_BENCH_BACKEND=gloo rehearses the N>1 path with several ranks on one GPU
        backend = os.environ.get("APD_BENCH_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        tdist.init_process_group(backend=backend)
        dist = (torch, tdist, backend)

    def barrier():
        if dist:
            torch, tdist, backend = dist
            tdist.barrier()
            if torch.cuda.is_available():
                torch.cuda.synchronize()

    import apd_abi as A

    W, H, N = args.width, args.height, args.n_src
    t0 = time.time()
    sc = make_scene(W, H, N, world, args.texture)
    t_scene = time.time() - t0
    n_views = len(sc.images)
    ref = rank % n_views
    ids = [ref] + [j for j, _ in sc.pairs[ref]][:N]

    lib = A.load_library()
    device = local_rank % max(1, lib.apd_device_count())
    if dist and dist[2] != "nccl":
        import torch
        if torch.cuda.is_available():
            torch.cuda.set_device(device)
    eng = A.Engine(device, lib)
    t0 = time.time()
    priors = first_init_priors(eng, sc, ids, N)
    t_priors = time.time() - t0
    arr = final_round_problem(sc, priors, ref, N)
    del priors
    weak_frac = float((arr.weak_info == A.WEAK).mean())

    exchange = exchange_timed = None
    per_rank = max(1, -(-args.scan_views // world))
    if dist:
        # this rank's view state as the scan runner packs it (depth, normal xyz, state, confidence),
        # from a finished run of its problem, on its device
        import scan_runner
        torch, tdist, backend = dist
        eng.set_problem(arr)
        eng.run()
        o = eng.results_device(W, H, f"cuda:{device}")
        state = scan_runner._pack(o.planes[..., 3], o.planes[..., :3], o.weak_info, o.confidence).contiguous()
        del o
        exchange, exchange_timed, wire_bytes = state_exchange(tdist, torch, state, world, per_rank)
        exchange(per_rank)  # (first use: communicator setup out of the timed region)
    elapsed, step_ms, pairs_ms = timed_fresh_iterations(eng, arr, args.steps, args.warmup, barrier, exchange, per_rank)
    PREP_LOG_HEADLINE = list(PREP_LOG)
    roof = weak_roofline(eng, args.steps, W, N)
    roof_strong_apd = strong_roofline(eng, W, N)
    eng.profile_reset(False)
    exch = None
    if dist:
        torch, tdist, backend = dist
        ex_ms = exchange_timed(5, per_rank)
        dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        mine = torch.tensor([elapsed, statistics.median(step_ms), ex_ms, pairs_ms], dtype=torch.float64, device=dev)
        every = [torch.zeros_like(mine) for _ in range(world)]
        tdist.all_gather(every, mine)
        every = [e.cpu().tolist() for e in every]
        elapsed = max(e[0] for e in every)
        loop_elapsed = max(e[0] - e[3] * 1e-3 for e in every)
        blocks = -(-args.steps // max(1, arr.params.max_iterations))
        exch = {"exchange_ms": round(max(e[2] for e in every), 3),
                "exchange_bytes_per_rank": wire_bytes,
                "exchange_bytes_per_px": scan_runner.WIRE_BYTES_PER_PX,
                "problems_per_rank_per_exchange": per_rank,
                "exchange_ms_basis": f"all-gather of {per_rank} states per rank",
                "exchanges_in_timed_region": -(-blocks // per_rank),
                "exchange_backend": backend,
                "rank_ms_per_step": [round(e[0] / args.steps * 1e3, 3) for e in every],
                "rank_iter_ms_median": [round(e[1], 3) for e in every],
                "note": "a scan pass on N ranks: every rank runs ceil(scan_views / N) problems (blocks of "
                        "fresh iterations), then one all-gather of their states (18 B/px wire format) inside "
                        "the timed region, as scan_runner.py ends every pass; exchange_ms = median of 5 "
                        "barrier-separated all-gathers of that many states, max over ranks"}
        del state

    n_gpus = world if dist else 1
    if not dist:
        loop_elapsed = elapsed - pairs_ms * 1e-3
    # the headline charges each pass's pair table to its iterations (timed_fresh_iterations);
    # the bare loop body is reported beside it
    value = n_gpus * W * H * args.steps / elapsed / 1e6
    value_loop = n_gpus * W * H * args.steps / loop_elapsed / 1e6

    line = None
    if rank == 0:
        e2e = end_to_end(eng, arr, sc, ref, W, H, N) if args.end_to_end else None
        del arr
        sa_pass = None
        if args.sa and n_gpus == 1:
            sa_pass = apd_pass_once(eng, sc, ref, N, f"C5's per-GPU workload: the {workload_name(W, H, N, True)} pass "
                                                   f"with SAM-style segment labels as the SA mask (APD.cu:464-530)", sa=True)
        del sc
        single = n_gpus == 1
        c2 = c2_first_init(eng, 6, 2) if (args.c2 and single) else None
        rich = None
        if args.rich and single and args.texture != "rich":
            rsc = make_scene(W, H, N, 1, "rich")
            rich = apd_pass_once(eng, rsc, 0, N, f"{workload_name(W, H, N, True)} pass on the texture-rich "
                                                  f"scene variant (synth texture='rich')")
            del rsc
        cpu = cpu1 = None
        if not args.no_cpu_baseline and single:
            cpu = cpu_baseline(eng, args.texture, N, W // 4, H // 4, args.cpu_threads, W, H)
            cpu1 = cpu_baseline(eng, args.texture, N, W // 16, H // 16, 1, W, H)
        name = workload_name(W, H, N, True)
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mpix/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (seeded piecewise-planar scan, apde-mvs_amd/synth.py, texture={args.texture}; "
                    f"no ETH3D data offline)",
            "config": {"workload": f"{name}: ETH3D-office-shaped scan, full-res {W}x{H}, 1 ref + {N} src views, "
                                   f"final-round REFINE_ITER pass (deformable PM + focal-weighted anchors + geom "
                                   f"consistency + impetus, rotate_time {arr_rt()}, priors from FIRST_INIT runs); "
                                   f"step = loop body APD.cu:2699-2708 (Strong B+R, RANSAC fit, Weak B+R) of "
                                   f"fresh runs; one ref view per GPU",
                       "width": W, "height": H, "n_src": N, "texture": args.texture,
                       "weak_frac": round(weak_frac, 4), "global_batch": n_gpus,
                       "parallelism": f"views{n_gpus}"},
            # `value` includes each pass's pair-table build (its HIP-event bracket on the ctx stream,
            # with RandomInitialization running beside it on a side stream: an upper bound of its
            # cost) spread over the pass's iterations; the loop body alone:
            "mpix_s_iter_loop": round(value_loop, 3),
            "pairs_ms_per_pass": round(pairs_ms / args.steps * max(1, arr_iters()), 3),
            "prepare_blocks": PREP_LOG_HEADLINE,
            "value_basis": "W*H*steps*n_gpus / (timed loop-body iterations + each pass's pair-table build "
                           "charged per iteration, max over ranks)",
            "multi_gpu": exch,
            "iter_ms_median": round(statistics.median(step_ms), 3),
            "iter_ms": [round(x, 2) for x in step_ms],
            "roofline": roof,
            "roofline_strong_sweep": roof_strong_apd,
            "roofline_depth_to_weak": e2e["roofline_depth_to_weak"] if e2e else None,
            "cpu_baseline": cpu,
            "cpu_baseline_1core": cpu1,
            "end_to_end": e2e,
            "c2_first_init": c2,
            "rich_texture": rich,
            "sa_pass": sa_pass,
            "scene_gen_s": round(t_scene, 2),
            "priors_s": round(t_priors, 2),
            "bench_wall_s": round(time.time() - t_start_all, 1),
        }
    eng.close()
    if dist:
        torch, tdist, backend = dist
        tdist.barrier()
        tdist.destroy_process_group()
    if line is not None:
        print(json.dumps(line), flush=True)


def arr_rt():
    return min(2 ** FINAL_ROUND, 4)


def arr_iters():
    return 3  # main.h:80 max_iterations (the final round's REFINE_ITER pass)


if __name__ == "__main__":
    main()
