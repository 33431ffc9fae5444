"""The fast-math oracle variant of the numerics-sensitivity study (tests/numerics_sensitivity.py,
profiles/r5_numerics_sensitivity.json) keeps building and stays the study it claims to be (CPU only):
liboracle_fm.so (ORACLE_FASTMATH: nvcc --use_fast_math's contraction, approximate division / sqrt /
exp, flush-to-zero, in spirit) is a different rounding of the same algorithm -- its outputs differ
from the parity contract's at the ulp level and diverge where PatchMatch's argmins amplify that, while
the ground-truth accuracy of both stays the same."""
import os
import subprocess

import numpy as np

import cases
import numerics_sensitivity as NS
import oracle_lib


def test_fastmath_variant_builds_and_differs():
    subprocess.run(["make", "-C", oracle_lib.ORACLE_DIR, "liboracle_fm.so"], check=True, capture_output=True)
    assert os.path.exists(oracle_lib.ORACLE_FM_SO)
    R = NS.Runner(4)
    sc = cases.scene(160, 120, 4)
    arr = cases.make_case("first_n4", R.run_c)
    c, f = R.run_c(arr), R.run_f(arr)
    m = NS.metrics(c, f, arr, sc.gt_depth[0])
    # the variant is active: most depths differ in their low bits
    assert m["depth_bit_identical_frac"] < 0.5
    # ... and it is a rounding change, not a different algorithm: the same scene quality, mostly the same
    # pixel states and view selections
    assert abs(m["gt_median_rel_err_contract"] - m["gt_median_rel_err_fastmath"]) < 1e-3
    assert m["pixel_state_agree_frac"] > 0.99 and m["selected_views_agree_frac"] > 0.9
    # the parity build itself is unchanged by the FDIV / FSQRT macros: equal to the committed fixture
    import golden_io
    for path in golden_io.fixtures():
        if os.path.basename(path) == "first_n4.npz":
            a2, expected = golden_io.load(path)
            assert all(v == 0 for v in golden_io.diff(expected, R.run_c(a2)).values())


def test_summary_shape():
    rec = {"pass": {"depth_within_1e-3_rel_frac": 0.8, "depth_bit_identical_frac": 0.2, "validity_mask_identical": True,
                    "validity_mask_agree_frac": 1.0, "pixel_state_identical": False, "pixel_state_agree_frac": 0.99,
                    "selected_views_agree_frac": 0.95, "depth_in_range_identical": True}}
    s = NS.summary([rec, rec])
    assert s["pass"]["cases"] == 2 and s["pass"]["validity_mask_identical_cases"] == 2
    assert np.isclose(s["pass"]["depth_within_1e-3_rel_frac_median"], 0.8)


def test_validity_mask_is_baselines_definition():
    """validity_mask_* is BASELINE.md §2's mask, depth > 0 and pixel state != UNKNOWN after the epilogue:
    a pixel whose state alone differs (UNKNOWN in one build, depth in range in both) breaks it, while
    depth_in_range_* (depth > 0 alone) does not see it."""
    import copy
    R = NS.Runner(4)
    arr = cases.make_case("first_n4", R.run_c)
    c = R.run_c(arr)
    f = copy.deepcopy(c)
    d, _, w = cases.epilogue(c, arr.params.depth_min, arr.params.depth_max)
    idx = np.argwhere((d > 0) & (w != 2))[:5]
    for y, x in idx:
        f.weak_info[y, x] = 2  # UNKNOWN
    m = NS.metrics(c, f, arr)
    assert m["depth_in_range_identical"] and not m["validity_mask_identical"]
    assert m["validity_mask_differing_pixels"] == len(idx) == 5
