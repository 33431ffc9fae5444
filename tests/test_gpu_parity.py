"""GPU parity: libapd_hip.so (through the C ABI) vs the CPU oracle, bit-exact on seeded inputs.

Tolerance: none — every float output (planes, costs) must match bit-for-bit (NaN == NaN), every
integer/byte output (PixelState, confidence, selected-view bitmask, view weights) exactly. The HIP
kernels and the oracle share one numerics contract (see oracle/apd_oracle.c header), so any
difference is a bug.
"""
import numpy as np
import pytest

import apd_abi as A
import cases
import oracle_lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def oracle():
    return oracle_lib.load()


@pytest.fixture(scope="module")
def engine():
    lib = A.load_library()
    if lib.apd_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    eng = A.Engine(0, lib)
    yield eng
    eng.close()


def run_hip(engine, arr):
    engine.set_problem(arr)
    engine.run()
    n_src = len(arr.images) - 1
    out = A.Outputs(arr.width, arr.height, n_src, max_weak=arr.width * arr.height)
    return engine.results(out)


@pytest.mark.parametrize("name", list(cases.CASES))
def test_bit_exact(name, oracle, engine):
    orun = lambda arr: oracle_lib.run(oracle, arr)
    arr = cases.make_case(name, orun)
    ref = oracle_lib.run(oracle, arr)
    got = run_hip(engine, arr)
    diffs = cases.compare(ref, got)
    assert all(v == 0 for v in diffs.values()), f"{name}: differing elements {diffs}"
    if arr.params.use_APD:
        wc = int(ref.weak_count[0])
        assert int(got.weak_count[0]) == wc
        assert np.array_equal(ref.anchors[:wc], got.anchors[:wc])


def test_reliable_curve_export(oracle, engine):
    """DepthToWeak's 61-sample cost curves (--export_curve, APD.cu:2188-2198) match bit-for-bit."""
    orun = lambda arr: oracle_lib.run(oracle, arr)
    arr = cases.make_case("refine_iter_geom", orun)
    arr.export_reliable_curve = True
    ref = oracle_lib.run(oracle, arr, want_curve=True)
    engine.set_problem(arr)
    engine.run()
    got = engine.results(A.Outputs(arr.width, arr.height, len(arr.images) - 1, want_curve=True))
    assert (ref.reliable_curve != 0).any()
    assert np.array_equal(ref.reliable_curve.view(np.uint32), got.reliable_curve.view(np.uint32))


def test_stages_equal_full_run(oracle, engine):
    """prepare + iteration(i) + finish must be the same computation as apd_run_patchmatch."""
    orun = lambda arr: oracle_lib.run(oracle, arr)
    arr = cases.make_case("first_n4", orun)
    full = run_hip(engine, arr)
    engine.set_problem(arr)
    engine.prepare()
    for i in range(arr.params.max_iterations):
        engine.iteration(i)
    engine.finish()
    engine.synchronize()
    staged = engine.results(A.Outputs(arr.width, arr.height, len(arr.images) - 1))
    assert all(v == 0 for v in cases.compare(full, staged).values())


def test_repeatable(oracle, engine):
    orun = lambda arr: oracle_lib.run(oracle, arr)
    arr = cases.make_case("first_n8", orun)
    a = run_hip(engine, arr)
    b = run_hip(engine, arr)
    assert all(v == 0 for v in cases.compare(a, b).values())


def test_errors_are_codes_not_exits(engine):
    sc = cases.scene(64, 48, 4)
    arr = cases.base_problem(sc, 0)
    arr.params.strong_radius = 7
    with pytest.raises(A.ApdError, match="APD_EINVAL"):
        engine.set_problem(arr)
    sc2 = cases.scene(64, 48, 4)
    arr2 = cases.base_problem(sc2, 0)
    arr2.images = list(arr2.images) * 9  # 36 images > MAX_IMAGES
    arr2.cameras = list(arr2.cameras) * 9
    with pytest.raises(A.ApdError, match="APD_ETOOMANYVIEWS"):
        engine.set_problem(arr2)
