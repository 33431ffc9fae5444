"""Numerics sensitivity of the PatchMatch path: how far the outputs move when the fp32 rounding contract
changes at the ulp level (SURVEY.md §7 hazard ii, §8c).

TEST INFRASTRUCTURE (it runs the CPU oracle only). The parity contract (oracle/liboracle.so, equal bit
for bit to the HIP kernels) rounds the reference's fp32 arithmetic one fixed way: -ffp-contract=off with
explicit fmaf at a fixed set of sites, IEEE division and sqrt, deterministic exp/sin/cos polynomials.
The reference is built with nvcc --use_fast_math (CMakeLists.txt:26): contraction of any a*b+c,
approximate division and square roots, __expf/__sinf/__cosf, flush-to-zero. liboracle_fm.so
(ORACLE_FASTMATH in oracle/apd_oracle.c) restates that build in spirit. Both run on the same inputs:

  pass   the same problem (inputs, priors, seed) through both builds: the sensitivity of one pass;
  chain  for problems whose priors come from earlier passes, the fast-math build also computes those
         priors (FIRST_INIT of every view), so differences compound as they would across a scan.

Per case the report gives depth agreement (bit-identical fraction, L1, the fraction of pixels within
the north star's 1e-3 relative), the validity mask (depth inside [depth_min, depth_max] after the
ProcessProblem epilogue, main.cpp:168-178) and pixel-state agreement, the selected-views agreement,
normal angles, and, where the synthetic scene has one, both builds' error against the ground truth.

    python tests/numerics_sensitivity.py [--out profiles/r5_numerics_sensitivity.json] [--quick]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [HERE, os.path.join(REPO, "apde-mvs_amd")]

import numpy as np  # noqa: E402

import apd_abi as A  # noqa: E402
import cases  # noqa: E402
import golden_io  # noqa: E402
import oracle_lib  # noqa: E402
import synth  # noqa: E402


def epilogue_depth(out, arr):
    d, n, w = cases.epilogue(out, arr.params.depth_min, arr.params.depth_max)
    return d, n, w


def flat_window_frac(arr, sel):
    """Fraction of the pixels in `sel` whose 6x6 step-2 reference window (clamped) is constant."""
    ys, xs = np.nonzero(sel)
    if ys.size == 0:
        return None
    img = np.asarray(arr.images[0], np.float32).reshape(arr.height, arr.width)
    off = np.arange(-5, 6, 2)
    yy = np.clip(ys[:, None, None] + off[None, :, None], 0, arr.height - 1)
    xx = np.clip(xs[:, None, None] + off[None, None, :], 0, arr.width - 1)
    w = img[yy, xx].reshape(ys.size, -1)
    return round(float((w.max(1) == w.min(1)).mean()), 6)


def metrics(c, f, arr, gt=None):
    dc, nc, wc = epilogue_depth(c, arr)
    df, nf, wf = epilogue_depth(f, arr)
    vc, vf = dc > 0, df > 0
    # BASELINE.md §2's validity mask: depth > 0 and pixel state not UNKNOWN (after the epilogue, which
    # also marks an out-of-range depth UNKNOWN)
    mc, mf = vc & (wc != A.UNKNOWN), vf & (wf != A.UNKNOWN)
    both = vc & vf
    hw = dc.size
    rel = np.abs(df[both] - dc[both]) / dc[both]
    within = np.zeros_like(vc)
    within[both] = rel <= 1e-3
    agree = within | (~vc & ~vf)  # both valid and within 1e-3, or both invalid
    dot = np.clip((nc * nf).sum(-1), -1.0, 1.0)[both]
    ang = np.degrees(np.arccos(dot)) if dot.size else np.zeros(1)
    r = {
        "pixels": int(hw),
        "depth_bit_identical_frac": round(float((dc.view(np.uint32) == df.view(np.uint32)).mean()), 6),
        "depth_l1": float(np.abs(df[both] - dc[both]).mean()) if both.any() else 0.0,
        "depth_l1_rel": float(rel.mean()) if rel.size else 0.0,
        "depth_within_1e-3_rel_frac": round(float(agree.mean()), 6),
        "depth_within_1e-3_rel_frac_of_valid": round(float(within[both].mean()) if both.any() else 1.0, 6),
        "validity_mask_identical": bool((mc == mf).all()),
        "validity_mask_agree_frac": round(float((mc == mf).mean()), 6),
        "validity_mask_differing_pixels": int((mc != mf).sum()),
        # of those, the pixels whose reference window (NCC-Old's 6x6 taps, step 2) is exactly flat: its
        # variance is 0 in IEEE arithmetic, the NCC 0/0, while an approximate reciprocal leaves a tiny
        # variance and a finite cost (the synthetic scenes' constant-intensity patches)
        "validity_mask_differing_flat_window_frac": flat_window_frac(arr, mc != mf),
        "validity_frac": round(float(mc.mean()), 6),
        "depth_in_range_identical": bool((vc == vf).all()),
        "depth_in_range_agree_frac": round(float((vc == vf).mean()), 6),
        "pixel_state_identical": bool((wc == wf).all()),
        "pixel_state_agree_frac": round(float((wc == wf).mean()), 6),
        "selected_views_agree_frac": round(float((c.selected_views == f.selected_views).mean()), 6),
        "normal_angle_deg_p50": round(float(np.percentile(ang, 50)), 6),
        "normal_angle_deg_p99": round(float(np.percentile(ang, 99)), 4),
        "weak_frac": round(float((wc == A.WEAK).mean()), 4),
    }
    if gt is not None:
        for tag, d in (("contract", dc), ("fastmath", df)):
            m = (gt > 0) & (d > 0)
            e = np.abs(d[m] - gt[m]) / gt[m]
            r[f"gt_median_rel_err_{tag}"] = round(float(np.median(e)), 6) if e.size else None
            r[f"gt_within_1pct_{tag}"] = round(float((e < 0.01).mean()), 4) if e.size else None
    return r


class Runner:
    def __init__(self, threads):
        self.c = oracle_lib.load()
        self.f = oracle_lib.load(oracle_lib.ORACLE_FM_SO)
        self.t = threads

    def run_c(self, arr):
        return oracle_lib.run(self.c, arr, self.t)

    def run_f(self, arr):
        return oracle_lib.run(self.f, arr, self.t)


def small_cases(R, names, out):
    for name in names:
        t0 = time.time()
        w, h, n, kind = cases.CASES[name]
        sc = cases.case_scene(name)
        arr = cases.make_case(name, R.run_c)
        c = R.run_c(arr)
        rec = {"case": name, "size": f"{w}x{h}", "n_src": n, "kind": kind,
               "pass": metrics(c, R.run_f(arr), arr, sc.gt_depth[0])}
        if not kind.startswith("first"):
            arr_f = cases.make_case(name, R.run_f)
            rec["chain"] = metrics(c, R.run_f(arr_f), arr, sc.gt_depth[0])
        rec["seconds"] = round(time.time() - t0, 1)
        out.append(rec)
        print(json.dumps(rec), flush=True)


def golden_cases(R, out):
    for path in golden_io.fixtures():
        arr, _ = golden_io.load(path)
        rec = {"case": "golden/" + os.path.basename(path), "size": f"{arr.width}x{arr.height}",
               "n_src": len(arr.images) - 1, "pass": metrics(R.run_c(arr), R.run_f(arr), arr)}
        out.append(rec)
        print(json.dumps(rec), flush=True)


def scene_case(R, label, sc, n, build, out):
    """A medium case whose priors are FIRST_INIT runs of every view: contract priors for `pass`, the
    fast-math build's own priors for `chain`."""
    t0 = time.time()
    pc = [R.run_c(cases.base_problem(sc, r, n)) for r in range(len(sc.images))]
    pf = [R.run_f(cases.base_problem(sc, r, n)) for r in range(len(sc.images))]
    first = cases.base_problem(sc, 0, n)
    rec = {"case": label, "size": f"{sc.width}x{sc.height}", "n_src": n,
           "first_init": metrics(pc[0], pf[0], first, sc.gt_depth[0])}
    arr = build(sc, pc, n)
    c = R.run_c(arr)
    rec["pass"] = metrics(c, R.run_f(arr), arr, sc.gt_depth[0])
    rec["chain"] = metrics(c, R.run_f(build(sc, pf, n)), arr, sc.gt_depth[0])
    rec["seconds"] = round(time.time() - t0, 1)
    out.append(rec)
    print(json.dumps(rec), flush=True)


def final_round(sc, priors, n):
    """bench.py's headline pass (main.cpp:336-352 with i = 3): REFINE_ITER, APD + focal + geom + impetus,
    rotate_time 4."""
    return cases.refine_problem(sc, priors, 0, n, state=A.REFINE_ITER, geom=True, apd=True, rotate_time=4,
                                ransac_threshold=0.01 - 3 * 0.00125, weak_peak_radius=4, use_impetus=1)


def tat_final(sc, priors, n):
    return cases.refine_problem(sc, priors, 0, n, state=A.REFINE_ITER, geom=True, apd=True, geom_factor=0.05,
                                rotate_time=4, ransac_threshold=0.01 - 2 * 0.00125, weak_peak_radius=4)


def summary(records):
    """Worst case and medians over the records' pass and chain entries."""
    s = {}
    for mode in ("pass", "chain"):
        rs = [r[mode] for r in records if mode in r]
        if not rs:
            continue
        s[mode] = {
            "cases": len(rs),
            "depth_within_1e-3_rel_frac_min": min(r["depth_within_1e-3_rel_frac"] for r in rs),
            "depth_within_1e-3_rel_frac_median": float(np.median([r["depth_within_1e-3_rel_frac"] for r in rs])),
            "depth_bit_identical_frac_median": float(np.median([r["depth_bit_identical_frac"] for r in rs])),
            "validity_mask_identical_cases": sum(r["validity_mask_identical"] for r in rs),
            "validity_mask_agree_frac_min": min(r["validity_mask_agree_frac"] for r in rs),
            "validity_mask_agree_frac_median": float(np.median([r["validity_mask_agree_frac"] for r in rs])),
            "depth_in_range_identical_cases": sum(r["depth_in_range_identical"] for r in rs),
            "pixel_state_identical_cases": sum(r["pixel_state_identical"] for r in rs),
            "pixel_state_agree_frac_min": min(r["pixel_state_agree_frac"] for r in rs),
            "selected_views_agree_frac_median": float(np.median([r["selected_views_agree_frac"] for r in rs])),
        }
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r6_numerics_sensitivity.json"))
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--quick", action="store_true", help="small cases only")
    args = ap.parse_args()
    R = Runner(args.threads)
    recs = []
    t0 = time.time()
    small_cases(R, list(cases.CASES), recs)
    golden_cases(R, recs)
    if not args.quick:
        scene_case(R, "756x504 N=8 APD + geom REFINE_ITER (test_gpu_fullsize medium case)",
                   synth.make_scene(756, 504, 8, seed=20251114), 8,
                   lambda sc, p, n: cases.refine_problem(sc, p, 0, n, state=A.REFINE_ITER, geom=True, apd=True), recs)
        scene_case(R, "756x504 N=10 final-round pass (bench headline pass, cpu_baseline scene)",
                   synth.make_scene(756, 504, 10, seed=20251114), 10, final_round, recs)
        scene_case(R, "480x264 N=10 TaT final pass (C4 quarter)", synth.make_scene(480, 264, 10, seed=20251114), 10,
                   tat_final, recs)
        scene_case(R, "480x264 N=10 SA final pass rt4 (C5 quarter)", synth.make_scene(480, 264, 10, seed=20251115), 10,
                   cases.c5_final_pass, recs)
    doc = {
        "what": "parity contract (liboracle.so == HIP bit for bit) vs a fast-math restatement (liboracle_fm.so: "
                "-ffp-contract=fast, a*rcp(b), rsqrt-based sqrt, __expf-style exp, libm sin/cos, FTZ/DAZ) "
                "of the reference's nvcc --use_fast_math build (CMakeLists.txt:26), same inputs and seeds",
        "north_star": "depth within 1e-3 relative, validity mask pixel-identical",
        "validity_mask": "BASELINE.md §2: depth > 0 and pixel state != UNKNOWN after the ProcessProblem epilogue "
                         "(main.cpp:168-178; validity_mask_*). depth_in_range_* is the weaker depth > 0 alone "
                         "(round 5's measure, nearly vacuous: hypotheses are drawn inside [depth_min, depth_max])",
        "summary": summary(recs),
        "cases": recs,
        "seconds": round(time.time() - t0, 1),
        "threads": args.threads,
    }
    with open(args.out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(doc["summary"], indent=1))


if __name__ == "__main__":
    main()
