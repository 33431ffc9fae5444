"""Seeded parity cases shared by the CPU (oracle/golden) and GPU (HIP vs oracle) tests.

Every case is a small synthetic scene (≤160x120, N≤31; C1's 640x480 N=4 FIRST_INIT with two
iterations) so the oracle finishes in seconds. The
prior-dependent states (REFINE_INIT / REFINE_ITER, geometric consistency, APD anchors, SA masks)
take their priors from an oracle FIRST_INIT pass over the neighbouring views, exactly the data flow
of main.cpp:306-367 (depths.bin / normals.bin / weak.bin / confidence.bin of the previous pass).
"""
from __future__ import annotations

import functools

import numpy as np

import apd_abi as A
import synth


@functools.lru_cache(maxsize=None)
def scene(w=160, h=120, n_src=4, seed=20251114, weak=True, texture="smooth", texture_scale=1.0):
    return synth.make_scene(w, h, n_src, seed=seed, weak_patches=weak, texture=texture, texture_scale=texture_scale)


def base_problem(sc, ref=0, n_src=None, **params):
    srcs = [j for j, _ in sc.pairs[ref]]
    if n_src is not None:
        srcs = srcs[:n_src]
    arr = A.scene_problem(sc, ref, srcs)
    for k, v in params.items():
        setattr(arr.params, k, v)
    return arr


def first_pass(oracle_run, sc, n_src=None):
    """Oracle FIRST_INIT pass over every view -> per-view (planes, weak, conf) after the epilogue."""
    outs = []
    for ref in range(len(sc.images)):
        arr = base_problem(sc, ref, n_src)
        out = oracle_run(arr)
        outs.append(out)
    return outs


def epilogue(out, dmin, dmax):
    """ProcessProblem's host epilogue (main.cpp:168-178)."""
    planes = out.planes
    d = planes[..., 3].copy()
    weak = out.weak_info.copy()
    bad = (d < dmin) | (d > dmax)
    d[bad] = 0
    weak[bad] = A.UNKNOWN
    return d, planes[..., :3].copy(), weak


def refine_problem(sc, priors, ref=0, n_src=None, state=A.REFINE_ITER, geom=True, apd=False, sa=False,
                   **params):
    """A REFINE_* problem for view `ref` whose priors come from `priors` (list of oracle outputs)."""
    arr = base_problem(sc, ref, n_src)
    ids = [ref] + [j for j, _ in sc.pairs[ref]][: (len(arr.images) - 1)]
    dmin, dmax = arr.params.depth_min, arr.params.depth_max
    deps = []
    for i in ids:
        d, _, _ = epilogue(priors[i], dmin, dmax)
        deps.append(d)
    d0, n0, w0 = epilogue(priors[ref], dmin, dmax)
    planes = np.concatenate([n0, d0[..., None]], -1).astype(np.float32)
    arr.depths = deps
    arr.init_planes = planes
    arr.params.state = state
    arr.params.geom_consistency = int(geom)
    arr.params.use_APD = int(apd)
    if apd:
        arr.weak_info = w0
        arr.confidence = priors[ref].confidence.copy()
        arr.params.rotate_time = 2
        arr.params.ransac_threshold = 0.01 - 1 * 0.00125
    if sa:
        arr.sa_mask = sc.labels[ref].copy()
        if sa == "zero_band":  # label 0 (no SA window) over a column band: waves mix both window forms
            arr.sa_mask[:, sc.width // 3: sc.width // 2] = 0
    for k, v in params.items():
        setattr(arr.params, k, v)
    return arr


CASES = {
    # name: (w, h, n_src, kind)
    "first_n4": (160, 120, 4, "first"),
    "first_n8": (128, 96, 8, "first"),
    "first_n3_odd": (96, 65, 3, "first"),      # odd H with H/2 % 16 == 0: last row never swept
    "first_n1": (64, 48, 1, "first"),
    "refine_iter_geom": (128, 96, 4, "geom"),
    "refine_init_apd": (128, 96, 4, "apd"),
    "refine_iter_apd_geom_sa": (128, 96, 4, "apd_geom_sa"),
    "first_n12": (96, 72, 12, "first"),           # view-major P2 in several rounds, 3 tasks per wave
    "refine_iter_n16_apd_geom": (80, 60, 16, "apd_geom"),
    "first_tiny": (21, 13, 2, "first"),          # smaller than a list tile / DepthToWeak tile, odd sizes
    "refine_init_apd_small": (40, 28, 2, "apd"),  # anchors and RANSAC where most searches leave the image
    "first_n31": (64, 48, 31, "first"),           # the reference's maximum (32 images): largest LDS tables
    "refine_iter_n31_apd_geom": (48, 40, 31, "apd_geom"),
    "first_n6_sa0": (112, 84, 6, "first_sa0"),          # SA quadrant windows in init + Strong sweep
    "refine_iter_geom_sa0": (128, 96, 4, "geom_sa0"),   # ... and in DepthToWeak / LocalRefine
    "refine_iter_apd_geom_sa0": (96, 72, 4, "apd_geom_sa0"),
    "refine_iter_apd_geom_rt4": (112, 84, 4, "apd_geom_rt4"),  # rotate_time 4 (rounds >= 2): 32 anchor slots
    # TaT_a / TaT_i datasets: geom_factor 0.05 (main.cpp:293-299), N = 10 as config C4, final round
    "refine_iter_tat_n10_apd_geom": (120, 66, 10, "apd_geom_tat"),
    "refine_init_tat_n10_geom": (120, 66, 10, "geom_tat_init"),
    # texture-rich scene variant (synth texture="rich"): fine detail, 30-50 % WEAK
    "first_n6_rich": (128, 96, 6, "first_rich"),
    "refine_iter_apd_geom_rich": (128, 96, 6, "apd_geom_rich"),
    # config C5's pass (final round with SAM edge priors): SA labels with a label-0 band, N = 10,
    # rotate_time 4 -- the image-wide pair table keyed by (window anchor, SA-filtered)
    "refine_iter_sa_n10_apd_geom_rt4": (144, 88, 10, "apd_geom_sa_rt4"),
    # config C1 (BASELINE configs[0]): 640x480, 1 ref + 4 src views, 2 iterations, FIRST_INIT
    "c1_first_n4_iter2": (640, 480, 4, "first_c1"),
    # the headline's exact parameter set (bench.py final_round_problem, main.cpp:336-352 with i = 3,
    # j = 0, ETH3D): REFINE_ITER, APD + focal + geom (geom_factor 0.2, main.cpp:297) + impetus, N = 10,
    # rotate_time 4, ransac_threshold 0.00625, weak_peak_radius 4, no SA
    "refine_iter_eth3d_final_n10": (240, 160, 10, "apd_geom_final"),
}


def c5_final_pass(sc, priors, n, ref=0):
    """main.cpp's last APD + geometric pass (i = 3: rotate_time 4) of a scan with SAM edge priors
    (APD.cpp:641-652): the reference view's labels, with a label-0 column band so that SA-filtered
    and unfiltered windows meet in one wave."""
    return refine_problem(sc, priors, ref, n, state=A.REFINE_ITER, geom=True, apd=True, sa="zero_band",
                          rotate_time=4, ransac_threshold=0.01 - 3 * 0.00125, weak_peak_radius=4)


def headline_pass(sc, priors, n, ref=0):
    """bench.py's headline pass: main.cpp's last round (i = 3), first geometric pass (j = 0) of an ETH3D
    scan without SA masks (main.cpp:336-352): rotate_time min(2^3, 4), ransac_threshold 0.01 - 3 *
    0.00125, weak_peak_radius max(4 - 2 j, 2), impetus on, geom_factor 0.2 (main.cpp:297)."""
    return refine_problem(sc, priors, ref, n, state=A.REFINE_ITER, geom=True, apd=True, rotate_time=4,
                          ransac_threshold=0.01 - 3 * 0.00125, weak_peak_radius=4, use_impetus=1, geom_factor=0.2)


def case_scene(name):
    w, h, n, kind = CASES[name]
    rich = kind.endswith("_rich")
    # the headline-parameter case renders C3's texture per pixel (synth texture_scale = 6048 / w), so
    # that most of its pixels are WEAK as at C3 (bench.py cpu_baseline samples the same way)
    ts = 6048.0 / w if kind == "apd_geom_final" else 1.0
    return scene(w, h, max(n, 4), texture="rich" if rich else "smooth", texture_scale=ts)


def make_case(name, oracle_run):
    w, h, n, kind = CASES[name]
    sc = case_scene(name)
    if kind in ("first", "first_rich"):
        return base_problem(sc, 0, n)
    if kind == "first_c1":
        return base_problem(sc, 0, n, max_iterations=2)
    if kind == "first_sa0":
        arr = base_problem(sc, 0, n)
        arr.sa_mask = sc.labels[0].copy()
        arr.sa_mask[:, w // 3: w // 2] = 0
        return arr
    priors = first_pass(oracle_run, sc, n)
    if kind == "geom":
        return refine_problem(sc, priors, 0, n, state=A.REFINE_ITER, geom=True)
    if kind == "apd":
        return refine_problem(sc, priors, 0, n, state=A.REFINE_INIT, geom=False, apd=True)
    if kind == "apd_geom_sa":
        return refine_problem(sc, priors, 0, n, state=A.REFINE_ITER, geom=True, apd=True, sa=True)
    if kind == "geom_sa0":
        return refine_problem(sc, priors, 0, n, state=A.REFINE_ITER, geom=True, sa="zero_band")
    if kind == "apd_geom_sa0":
        return refine_problem(sc, priors, 0, n, state=A.REFINE_ITER, geom=True, apd=True, sa="zero_band")
    if kind == "apd_geom_sa_rt4":
        return c5_final_pass(sc, priors, n)
    if kind == "apd_geom_final":
        return headline_pass(sc, priors, n)
    if kind == "apd_geom_rt4":
        return refine_problem(sc, priors, 0, n, state=A.REFINE_ITER, geom=True, apd=True, rotate_time=4)
    if kind in ("apd_geom", "apd_geom_rich"):
        return refine_problem(sc, priors, 0, n, state=A.REFINE_ITER, geom=True, apd=True)
    if kind == "apd_geom_tat":  # main.cpp round 3, geometric pass j = 1 of a TaT scan
        return refine_problem(sc, priors, 0, n, state=A.REFINE_ITER, geom=True, apd=True, geom_factor=0.05,
                              rotate_time=4, ransac_threshold=0.01 - 3 * 0.00125, weak_peak_radius=2)
    if kind == "geom_tat_init":  # REFINE_INIT with geometric consistency (the `apd` binary's 2-round path)
        return refine_problem(sc, priors, 0, n, state=A.REFINE_INIT, geom=True, geom_factor=0.05)
    raise KeyError(kind)


FIELDS = ("planes", "costs", "weak_info", "confidence", "selected_views", "view_weights")


def compare(a, b, fields=FIELDS):
    """Bit-level comparison; returns {field: number of differing elements} (NaN == NaN)."""
    diffs = {}
    for f in fields:
        x, y = getattr(a, f), getattr(b, f)
        if x.dtype.kind == "f":
            xb = x.view(np.uint32)
            yb = y.view(np.uint32)
            same = (xb == yb) | (np.isnan(x) & np.isnan(y))
        else:
            same = x == y
        diffs[f] = int((~same).sum())
    return diffs
