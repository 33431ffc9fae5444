"""Benchmark: Mpix/s per PatchMatch iteration on the BASELINE.json configs[1] workload.

Workload (BASELINE.md §3 "C2"): a synthetic ETH3D-office-shaped scan at half resolution, 3024x2016,
one reference view + 8 source views, FIRST_INIT pass (geometric consistency off, APD off). A "step" is
one iteration of the sweep loop body (APD.cu:2699-2708: Black + Red Strong checkerboard kernels) over
the whole reference view; the view is uploaded and initialised (RandomInitialization) before the timed
region, so inputs are resident in HBM. value = W*H*steps summed over ranks / max-over-ranks time.

Multi-GPU (weak scaling): one process per GPU (torch.distributed.run), each rank runs its own reference
view of the scan (the scan's views are independent in a FIRST_INIT pass); the only collectives are the
timing barrier and a max-reduction of the elapsed time (no data-path collective).

Besides the headline line the JSON carries:
  roofline      dominant kernel (k_sweep_strong): algorithmic FP32 flops per launch (SURVEY.md §8d:
                1446 flop per NCC-Old evaluation x evaluations actually issued) / its mean launch time
                from HIP events on the engine stream, against the FP32 peak; HBM bytes from the latest
                rocprofv3 PMC summary under profiles/ when present.
  cpu_baseline  the C oracle (oracle/liboracle.so, OpenMP) on a bounded sample: the same scene rendered
                at 756x504 (same cameras/texture statistics, same N), one sweep iteration.
  apd_pass      (rank 0) the same metric for an APD + geometric-consistency pass (main.cpp rounds >= 1)
                on the same view, priors from FIRST_INIT runs of every view of the scene.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402

METRIC = "Mpix/s per PatchMatch iteration (ref view, N src) at 1/2/4/8 GPU; depth L1 vs ref"
FLOP_PER_NCC_OLD = 36 * 36 + 150  # 36 samples x 36 flop + homography/finalise
PEAK_FP32_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector (= FP32 matrix) peak
PEAK_HBM_GBS = 8000.0


def strong_evaluations(W: int, H: int, n_src: int, colour: int, row_limit: int) -> int:
    """Upper bound on the NCC-Old evaluations of one Strong sweep launch over a colour: per pixel
    (valid adaptive-checkerboard neighbours + current + 5 refinement candidates) x N views. The
    refinement NCCs of views with sampled weight 0 are skipped by the kernel, so the device count
    (apd_profile_evaluations) is lower; roofline.achieved uses the device count."""
    ys = np.arange(row_limit)[:, None]
    xs = np.arange(W)[None, :]
    mask = ((xs + ys) & 1) == colour
    flags = ((ys > 2).astype(int) + (ys < H - 3) + (xs > 2) + (xs < W - 3) + (ys > 0) + (ys < H - 1)
             + (xs > 0) + (xs < W - 1))
    per_px = flags + 6
    return int((per_px * mask).sum()) * n_src


def latest_pmc(kernel: str, W: int, n_src: int):
    """The newest (by round/session file name) PMC summary under profiles/ for this kernel and shape.
    Other PMC files (counter studies of other shapes or blocks) are skipped, not taken as the latest."""
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc*.json")), reverse=True):
        try:
            pmc = json.load(open(f))
        except Exception:
            continue
        if (isinstance(pmc, dict) and str(pmc.get("kernel", "")).startswith(kernel)
                and pmc.get("width") == W and pmc.get("n_src") == n_src
                and pmc.get("hbm_bytes_per_launch") is not None):
            return pmc
    return None


def cpu_baseline(scene_args, n_src, threads):
    import oracle_lib
    import synth
    import apd_abi as A

    w, h = 756, 504
    sc = synth.make_scene(w, h, n_src, **scene_args)
    arr = A.scene_problem(sc, 0, [j for j, _ in sc.pairs[0]][:n_src])
    lib = oracle_lib.load()
    import ctypes as C
    pb = arr.build()
    times = (C.c_double * 3)()
    st = lib.oracle_time_iterations(C.byref(pb), 1, threads, times)
    if st != 0:
        return None
    t_iter = times[1]
    return {"value": round(w * h / t_iter / 1e6, 4), "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": f"oracle (C restatement, OpenMP) on the same synthetic scene rendered at {w}x{h}, N={n_src}, "
                      f"FIRST_INIT, one sweep iteration (t_iter={t_iter:.2f}s; prepare {times[0]:.2f}s untimed)"}


def apd_pass(eng, sc, ref, N):
    """One REFINE_ITER problem with APD (deformable NCC, focal weights, anchors) and geometric
    consistency on -- what main.cpp runs in rounds >= 1 -- on the same scene, priors from FIRST_INIT
    runs of every view (the data flow of round 0). Per-iteration Mpix/s as the headline metric
    (loop body = Strong B+R, RANSAC fit, candidate costs, Weak B+R), median over the 3 iterations."""
    import apd_abi as A
    import cases
    import statistics
    W, H = sc.width, sc.height
    priors = []
    for r in range(len(sc.images)):
        arr = A.scene_problem(sc, r, [j for j, _ in sc.pairs[r]][:N], seed=0x5EED ^ r)
        eng.set_problem(arr)
        eng.run()
        priors.append(eng.results(A.Outputs(W, H, N)))
    arr = cases.refine_problem(sc, priors, ref, N, state=A.REFINE_ITER, geom=True, apd=True)
    eng.set_problem(arr)
    eng.run()
    tm = eng.timing()
    iters = list(tm.iter_ms)[: tm.iterations]
    return {"mpix_s_iter": round(W * H / (statistics.median(iters) * 1e-3) / 1e6, 3),
            "iter_ms": [round(x, 2) for x in iters], "run_patchmatch_ms": round(tm.total_ms, 2),
            "mpix_s_end_to_end": round(W * H * tm.iterations / (tm.total_ms * 1e-3) / 1e6, 3),
            "anchors_ms": round(tm.anchors_ms, 2), "init_ms": round(tm.init_ms, 2), "sweep_ms": round(tm.sweep_ms, 2),
            "post_ms": round(tm.post_ms, 2), "weak_frac": round(float((arr.weak_info == A.WEAK).mean()), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--width", type=int, default=3024)
    ap.add_argument("--height", type=int, default=2016)
    ap.add_argument("--n-src", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    ap.add_argument("--end-to-end", type=int, default=1, help="also time one full RunPatchMatch (0/1)")
    ap.add_argument("--apd-pass", type=int, default=1,
                    help="also time one APD + geometric-consistency pass (REFINE_ITER, rounds >= 1) (0/1)")
    args = ap.parse_args()

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

    import apd_abi as A
    import synth

    W, H, N = args.width, args.height, args.n_src
    scene_args = dict(seed=20251114)
    t0 = time.time()
    sc = synth.make_scene(W, H, max(N, world), **scene_args)
    t_scene = time.time() - t0
    n_views = len(sc.images)
    ref = rank % n_views
    srcs = [j for j, _ in sc.pairs[ref]][:N]
    arr = A.scene_problem(sc, ref, srcs, seed=0x5EED ^ ref)

    lib = A.load_library()
    device = local_rank % max(1, lib.apd_device_count())
    eng = A.Engine(device, lib)
    eng.set_problem(arr)
    eng.prepare()
    eng.synchronize()
    iters = arr.params.max_iterations
    for s in range(args.warmup):
        eng.iteration(s % iters)
    eng.synchronize()

    def barrier():
        if dist:
            torch, tdist, backend = dist
            tdist.barrier()
            if torch.cuda.is_available():
                torch.cuda.synchronize()

    eng.profile_reset(True)
    barrier()
    eng.synchronize()
    t_start = time.perf_counter()
    for s in range(args.steps):
        eng.iteration(s % iters)
    eng.synchronize()
    t_end = time.perf_counter()
    barrier()
    elapsed = t_end - t_start
    sweep_ms, launches, sweep_px = eng.profile_query()
    ncc_evals = eng.profile_evaluations()
    eng.profile_reset(False)
    if dist:
        torch, tdist, backend = dist
        dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())

    n_gpus = world if dist else 1
    value = n_gpus * W * H * args.steps / elapsed / 1e6

    # dominant kernel roofline (k_sweep_strong): flops of the NCC-Old evaluations the launches actually
    # issued (counted on the device), per launch; the static upper bound is kept beside it
    hh = H // 2
    row_limit = min(H, 32 * ((hh + 15) // 16))
    evals_bound = strong_evaluations(W, H, N, 0, row_limit) + strong_evaluations(W, H, N, 1, row_limit)
    flop_per_launch = ncc_evals / max(launches, 1) * FLOP_PER_NCC_OLD
    launch_ms = sweep_ms / max(launches, 1)
    achieved_tf = flop_per_launch / (launch_ms * 1e-3) / 1e12
    bytes_per_launch = (W * H / 2) * (4 * (N + 1) + 80)  # = 116 B/px at N=8
    pmc = latest_pmc("k_sweep_strong", W, N)
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None

    line = None
    if rank == 0:
        e2e = None
        if args.end_to_end:
            eng.set_problem(arr)
            t1 = time.perf_counter()
            eng.run()
            t2 = time.perf_counter()
            tm = eng.timing()
            out = eng.results(A.Outputs(W, H, N))
            gt = sc.gt_depth[ref]
            d = out.planes[..., 3]
            m = (gt > 0) & (out.weak_info != A.UNKNOWN)
            rel = np.abs(d[m] - gt[m]) / gt[m]
            e2e = {"run_patchmatch_ms": round(tm.total_ms, 3), "host_wall_ms": round((t2 - t1) * 1e3, 3),
                   "mpix_s_end_to_end": round(W * H * iters / (tm.total_ms * 1e-3) / 1e6, 3),
                   "init_ms": round(tm.init_ms, 3), "sweep_ms": round(tm.sweep_ms, 3),
                   "post_ms": round(tm.post_ms, 3),
                   "iter_ms": [round(x, 3) for x in list(tm.iter_ms)[:iters]],
                   "gt_median_rel_depth_err": round(float(np.median(rel)), 5),
                   "gt_frac_within_1pct": round(float((rel < 0.01).mean()), 4)}
        apd = apd_pass(eng, sc, ref, N) if args.apd_pass else None
        cpu = None if args.no_cpu_baseline else cpu_baseline(scene_args, N, args.cpu_threads)
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
            "data": "synthetic (seeded piecewise-planar scan, apde-mvs_amd/synth.py; no ETH3D data offline)",
            "config": {"workload": "C2: ETH3D-office-shaped scan, half-res 3024x2016, 1 ref + 8 src views, "
                                   "FIRST_INIT sweep iteration (geom off, APD off), one ref view per GPU",
                       "width": W, "height": H, "n_src": N, "global_batch": n_gpus, "parallelism": f"views{n_gpus}"},
            "roofline": {"bound": "mfma", "achieved": round(achieved_tf, 3), "peak": PEAK_FP32_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved_tf / PEAK_FP32_TFLOPS, 4),
                         "traffic": traffic,
                         "kernel": "k_sweep_strong",
                         "note": "VALU-FP32 gather/stencil kernel (no matrix work): priced against the FP32 "
                                 "peak, which on gfx950 is the same 157.3 TF for VALU and f32 MFMA",
                         "launch_ms": round(launch_ms, 4), "launches": launches,
                         "flop_per_launch": flop_per_launch,
                         "ncc_evals_per_launch": round(ncc_evals / max(launches, 1)),
                         "ncc_evals_bound_per_launch": evals_bound // 2,
                         "hbm_algorithmic_gbs": round(bytes_per_launch / (launch_ms * 1e-3) / 1e9, 2),
                         "hbm_peak_gbs": PEAK_HBM_GBS},
            "cpu_baseline": cpu,
            "end_to_end": e2e,
            "apd_pass": apd,
            "scene_gen_s": round(t_scene, 2),
        }
    eng.close()
    if dist:
        torch, tdist, backend = dist
        tdist.barrier()
        tdist.destroy_process_group()
    if line is not None:
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
