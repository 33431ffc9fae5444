"""GPU checks beyond the small parity cases of test_gpu_parity.py.

* medium size, bit-exact against the CPU oracle: a 1512x1008 FIRST_INIT problem with N = 8 (the bench
  scene rendered at half scale) and a 756x504 APD + geometric-consistency REFINE_ITER problem with N = 8,
  whose priors are the HIP engine's own FIRST_INIT outputs of the neighbouring views (priors are
  inputs: both sides read the same ones);
* full size (BASELINE.json configs[1]: 3024x2016, N = 8), where the oracle would take minutes, through
  properties that do not depend on the size: the result is a pure function of the inputs and the seed
  (two runs are bit-identical), it does not depend on how pixels are dealt to workgroups (list tile
  width 8 vs 16) nor on the source-texel storage (fp16 vertical pairs vs fp32 quads), and the depth
  agrees with the synthetic scene's ground truth (median relative error < 0.2 %, >= 60 % of the
  pixels within 1 %; the bench measures 0.07 % and 71 %).
Tolerance: none for the comparisons (bit-for-bit, NaN == NaN); the ground-truth bounds are quality
floors, not parity claims.
"""
import os

import numpy as np
import pytest

import apd_abi as A
import cases
import oracle_lib
import synth

pytestmark = pytest.mark.gpu

FULL_W, FULL_H, N = 3024, 2016, 8


@pytest.fixture(scope="module")
def lib():
    lib = A.load_library()
    if lib.apd_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return lib


@pytest.fixture(scope="module")
def engine(lib):
    eng = A.Engine(0, lib)
    yield eng
    eng.close()


@pytest.fixture(scope="module")
def engine_tw16(lib):
    """Second context whose sweep lists use 16-wide tiles (different workgroup composition)."""
    os.environ["APD_TILE_W"] = "16"
    try:
        eng = A.Engine(0, lib)
    finally:
        os.environ.pop("APD_TILE_W", None)
    yield eng
    eng.close()


@pytest.fixture(scope="module")
def full_scene():
    return synth.make_scene(FULL_W, FULL_H, N, seed=20251114)


def run(eng, arr, f32=False):
    if f32:
        os.environ["APD_TEX_F32"] = "1"
    try:
        eng.set_problem(arr)
    finally:
        os.environ.pop("APD_TEX_F32", None)
    eng.run()
    return eng.results(A.Outputs(arr.width, arr.height, len(arr.images) - 1, max_weak=arr.width * arr.height))


def assert_same(a, b, what):
    d = cases.compare(a, b)
    assert not any(d.values()), f"{what}: differing elements {d}"


def hip_priors(eng, sc, n):
    return [run(eng, cases.base_problem(sc, r, n)) for r in range(len(sc.images))]


def test_medium_first_init_bit_exact(engine):
    sc = synth.make_scene(1512, 1008, N, seed=20251114)
    arr = cases.base_problem(sc, 0, N)
    ref = oracle_lib.run(oracle_lib.load(), arr, 16)
    assert_same(ref, run(engine, arr), "1512x1008 FIRST_INIT")


def test_medium_apd_pass_bit_exact(engine):
    sc = synth.make_scene(756, 504, N, seed=20251114)
    arr = cases.refine_problem(sc, hip_priors(engine, sc, N), 0, N, state=A.REFINE_ITER, geom=True, apd=True)
    assert (arr.weak_info == A.WEAK).any()
    ref = oracle_lib.run(oracle_lib.load(), arr, 16)
    got = run(engine, arr)
    assert_same(ref, got, "756x504 APD + geom REFINE_ITER")
    wc = int(ref.weak_count[0])
    assert int(got.weak_count[0]) == wc


def test_fullsize_first_init_properties(engine, engine_tw16, full_scene):
    arr = cases.base_problem(full_scene, 0, N)
    a = run(engine, arr)
    assert_same(a, run(engine, arr), "repeat run")
    assert_same(a, run(engine_tw16, arr), "16-wide list tiles")
    assert_same(a, run(engine, arr, f32=True), "fp32 quad texels")
    gt = full_scene.gt_depth[0]
    d = a.planes[..., 3]
    m = (gt > 0) & (a.weak_info != A.UNKNOWN)
    rel = np.abs(d[m] - gt[m]) / gt[m]
    assert m.mean() > 0.5
    assert float(np.median(rel)) < 2e-3
    assert float((rel < 0.01).mean()) > 0.6


def test_fullsize_apd_pass_properties(engine, engine_tw16, full_scene):
    priors = hip_priors(engine, full_scene, N)
    arr = cases.refine_problem(full_scene, priors, 0, N, state=A.REFINE_ITER, geom=True, apd=True)
    a = run(engine, arr)
    assert int(a.weak_count[0]) > 0
    assert_same(a, run(engine, arr), "repeat APD run")
    assert_same(a, run(engine_tw16, arr), "16-wide list tiles (APD)")
    assert_same(a, run(engine, arr, f32=True), "fp32 quad texels (APD)")


# ---- configs C4 and C3 at their real shapes (BASELINE.json configs[3] / configs[2])

def slim_priors(eng, sc, n, ids):
    """FIRST_INIT outputs of the views in `ids` (planes, pixel states, confidence only: at 6048x4032
    a full Outputs per view would hold ~0.9 GB)."""
    out = [None] * len(sc.images)
    for r in ids:
        eng.set_problem(cases.base_problem(sc, r, n))
        eng.run()
        o = A.Outputs.__new__(A.Outputs)
        o.planes = np.zeros((sc.height, sc.width, 4), np.float32)
        o.weak_info = np.zeros((sc.height, sc.width), np.uint8)
        o.confidence = np.zeros((sc.height, sc.width), np.uint8)
        s = A.ApdOutputs()
        s.planes = A._ptr(o.planes, A.C.c_float)
        s.weak_info = A._ptr(o.weak_info, A.C.c_uint8)
        s.confidence = A._ptr(o.confidence, A.C.c_uint8)
        eng._check(eng.lib.apd_get_results(eng.ctx, A.C.byref(s)), "apd_get_results")
        out[r] = o
    return out


SLIM = ("planes", "costs", "weak_info", "confidence", "selected_views")


def run_slim(eng, arr):
    eng.set_problem(arr)
    eng.run()
    o = A.Outputs.__new__(A.Outputs)
    o.planes = np.zeros((arr.height, arr.width, 4), np.float32)
    o.costs = np.zeros((arr.height, arr.width), np.float32)
    o.weak_info = np.zeros((arr.height, arr.width), np.uint8)
    o.confidence = np.zeros((arr.height, arr.width), np.uint8)
    o.selected_views = np.zeros((arr.height, arr.width), np.uint32)
    o.weak_count = np.zeros(1, np.int32)
    s = A.ApdOutputs()
    for f, t in (("planes", A.C.c_float), ("costs", A.C.c_float), ("weak_info", A.C.c_uint8),
                 ("confidence", A.C.c_uint8), ("selected_views", A.C.c_uint32), ("weak_count", A.C.c_int32)):
        setattr(s, f, A._ptr(getattr(o, f), t))
    eng._check(eng.lib.apd_get_results(eng.ctx, A.C.byref(s)), "apd_get_results")
    return o


def assert_same_slim(a, b, what):
    d = cases.compare(a, b, SLIM)
    assert not any(d.values()), f"{what}: differing elements {d}"


def gt_floor(sc, out, ref=0, median=2e-3, within=0.6):
    gt = sc.gt_depth[ref]
    d = out.planes[..., 3]
    m = (gt > 0) & (out.weak_info != A.UNKNOWN)
    rel = np.abs(d[m] - gt[m]) / gt[m]
    assert m.mean() > 0.5
    assert float(np.median(rel)) < median, float(np.median(rel))
    assert float((rel < 0.01).mean()) > within, float((rel < 0.01).mean())


def tat_final_pass(sc, priors, n):
    """main.cpp's last geometric pass of a TaT scan (geom_factor 0.05, main.cpp:293-299)."""
    return cases.refine_problem(sc, priors, 0, n, state=A.REFINE_ITER, geom=True, apd=True, geom_factor=0.05,
                                rotate_time=4, ransac_threshold=0.01 - 2 * 0.00125, weak_peak_radius=4)


def test_c4_quarter_tat_bit_exact(engine):
    """C4's scene at a quarter of its size (480x264, N = 10, TaT geom_factor 0.05), final-round APD +
    geom pass, bit-exact against the oracle."""
    sc = synth.make_scene(480, 264, 10, seed=20251114)
    priors = slim_priors(engine, sc, 10, range(len(sc.images)))
    arr = tat_final_pass(sc, priors, 10)
    assert (arr.weak_info == A.WEAK).any()
    ref = oracle_lib.run(oracle_lib.load(), arr, 16)
    got = run(engine, arr)
    assert_same(ref, got, "480x264 N=10 TaT APD + geom")


def test_c4_fullsize_tat_properties(engine, engine_tw16):
    """Config C4 (T&T Family shape, 1920x1056, N = 10, TaT geom_factor 0.05): the FIRST_INIT pass and
    the final-round APD + geometric pass; repeat-run identity, list-tile independence, fp32 texels,
    ground-truth floors."""
    sc = synth.make_scene(1920, 1056, 10, seed=20251114)
    first = cases.base_problem(sc, 0, 10)
    f = run_slim(engine, first)
    assert_same_slim(f, run_slim(engine_tw16, first), "C4 FIRST_INIT, 16-wide list tiles")
    gt_floor(sc, f)
    priors = slim_priors(engine, sc, 10, range(len(sc.images)))
    arr = tat_final_pass(sc, priors, 10)
    a = run_slim(engine, arr)
    assert int(a.weak_count[0]) > 0
    assert_same_slim(a, run_slim(engine, arr), "C4 repeat APD run")
    assert_same_slim(a, run_slim(engine_tw16, arr), "C4 16-wide list tiles (APD)")
    os.environ["APD_TEX_F32"] = "1"
    try:
        b = run_slim(engine, arr)
    finally:
        os.environ.pop("APD_TEX_F32", None)
    assert_same_slim(a, b, "C4 fp32 quad texels (APD)")
    assert np.isfinite(a.planes[..., 3]).all()
    gt_floor(sc, a)


def test_c3_fullsize_apd_properties(engine, engine_tw16):
    """Config C3 at its real shape (6048x4032, N = 10), the final-round APD + focal + geometric
    REFINE_ITER pass (the bench's headline problem): repeat-run identity, list-tile independence,
    the DepthToWeak -> LocalRefine hand-over (21.5 GB, > 2^31 elements) == LocalRefine evaluating
    every sample itself (APD_NO_LR_HANDOVER=1), finite depths, ground-truth floors."""
    sc = synth.make_scene(6048, 4032, 10, seed=20251114)
    priors = slim_priors(engine, sc, 10, range(len(sc.images)))
    arr = cases.refine_problem(sc, priors, 0, 10, state=A.REFINE_ITER, geom=True, apd=True, rotate_time=4,
                               ransac_threshold=0.01 - 3 * 0.00125, weak_peak_radius=4)
    del priors
    a = run_slim(engine, arr)
    assert int(a.weak_count[0]) > 0
    assert_same_slim(a, run_slim(engine, arr), "C3 repeat run")
    assert_same_slim(a, run_slim(engine_tw16, arr), "C3 16-wide list tiles")
    os.environ["APD_NO_LR_HANDOVER"] = "1"
    try:
        eng = A.Engine(0, engine.lib)
    finally:
        os.environ.pop("APD_NO_LR_HANDOVER", None)
    try:
        assert_same_slim(a, run_slim(eng, arr), "C3 LocalRefine without the hand-over")
    finally:
        eng.close()
    assert np.isfinite(a.planes[..., 3]).all()
    gt_floor(sc, a)


# ---- config C5's per-GPU workload (BASELINE.json configs[4]): the final-round APD pass with SAM edge
# priors (SA labels, APD.cu:464-530, 664-719) at full resolution

def test_c5_quarter_sa_bit_exact(engine):
    """C5's pass at 480x264, N = 10 (SA labels with a label-0 band, rotate_time 4), bit-exact against
    the oracle."""
    sc = synth.make_scene(480, 264, 10, seed=20251115)
    priors = slim_priors(engine, sc, 10, range(len(sc.images)))
    arr = cases.c5_final_pass(sc, priors, 10)
    assert (arr.weak_info == A.WEAK).any() and (arr.sa_mask > 0).any() and (arr.sa_mask == 0).any()
    ref = oracle_lib.run(oracle_lib.load(), arr, 16)
    got = run(engine, arr)
    assert_same(ref, got, "480x264 N=10 SA APD + geom rt4")


def test_c5_fullsize_sa_properties(engine, engine_tw16):
    """C5's pass at its real shape (6048x4032, N = 10, SA labels with a label-0 band, rotate_time 4):
    repeat-run identity, list-tile independence, fp32 texels, LocalRefine without the hand-over, the
    Weak sweep evaluating the anchor candidates itself (APD_NO_CAND_PAIRS=1) == the SA-keyed pair
    table, finite depths, ground-truth floors."""
    sc = synth.make_scene(6048, 4032, 10, seed=20251115)
    priors = slim_priors(engine, sc, 10, range(len(sc.images)))
    arr = cases.c5_final_pass(sc, priors, 10)
    del priors
    assert (arr.sa_mask > 0).mean() > 0.5
    a = run_slim(engine, arr)
    assert int(a.weak_count[0]) > 0
    assert_same_slim(a, run_slim(engine, arr), "C5 repeat run")
    assert_same_slim(a, run_slim(engine_tw16, arr), "C5 16-wide list tiles")
    for var, what in (("APD_TEX_F32", "fp32 quad texels"), ("APD_NO_LR_HANDOVER", "LocalRefine without the hand-over"),
                      ("APD_NO_CAND_PAIRS", "anchor candidates in the sweep")):
        os.environ[var] = "1"
        try:
            eng = A.Engine(0, engine.lib)
            try:
                assert_same_slim(a, run_slim(eng, arr), "C5 " + what)
            finally:
                eng.close()
        finally:
            os.environ.pop(var, None)
    assert np.isfinite(a.planes[..., 3]).all()
    gt_floor(sc, a)
