"""CPU: the oracle's access-set checking mode (oracle/liboracle_rc.so, -DORACLE_RACECHECK).

SURVEY §5 asks for "a CPU oracle with a per-colour write-set ∩ read-set = ∅ assertion mode": the
reference runs every pixel of a launch concurrently (one CUDA thread per pixel; the checkerboard
colours, the in-place filter / DepthToWeak / LocalRefine / confidence tiles), so its result is
well defined only if no pixel of a launch reads or writes a state element another pixel of the same
launch writes. The checking build records, per launch (FOR_ALL / FOR_COLOUR phase), the writer and
the readers of every element of plane / cost / selected views / view weights / weak / confidence /
fit / reliable / nearest / anchors / curve / anchors map, and counts every cross-task write-read or
write-write. Checked here over the full schedule of the parity cases: zero conflicts, and the
instrumented build computes the same outputs as the normal one. The negative control runs the two
colours of each checkerboard as one launch: that must be caught.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import apd_abi as A
import cases
import oracle_lib

RC_SO = os.path.join(oracle_lib.ORACLE_DIR, "liboracle_rc.so")


@pytest.fixture(scope="module")
def oracle():
    return oracle_lib.load()


@pytest.fixture(scope="module")
def rc():
    subprocess.run(["make", "-C", oracle_lib.ORACLE_DIR, "liboracle_rc.so"], check=True, capture_output=True)
    lib = C.CDLL(RC_SO)
    lib.oracle_run_patchmatch.restype = C.c_int
    lib.oracle_run_patchmatch.argtypes = [C.POINTER(A.ApdProblem), C.POINTER(A.ApdOutputs), C.c_int,
                                          C.POINTER(C.c_double)]
    lib.oracle_racecheck_report.restype = C.c_int64
    lib.oracle_racecheck_report.argtypes = [C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.c_char_p, C.c_int]
    return lib


def report(rc, merge_next=0):
    ph, acc = C.c_int64(), C.c_int64()
    buf = C.create_string_buffer(320)
    n = rc.oracle_racecheck_report(merge_next, C.byref(ph), C.byref(acc), buf, len(buf))
    return n, ph.value, acc.value, buf.value.decode()


CHECKED = ["first_n4", "first_tiny", "first_n3_odd", "refine_iter_geom", "refine_init_apd", "refine_iter_apd_geom_sa",
           "refine_iter_apd_geom_sa0", "refine_init_apd_small", "refine_iter_apd_geom_rt4",
           "refine_iter_tat_n10_apd_geom"]


@pytest.mark.parametrize("name", CHECKED)
def test_no_cross_pixel_access_within_a_launch(name, oracle, rc):
    arr = cases.make_case(name, lambda a: oracle_lib.run(oracle, a))
    report(rc)  # reset
    got = oracle_lib.run(rc, arr, nthreads=1, want_curve=True)
    n, phases, accesses, first = report(rc)
    # every launch of the schedule was checked: 3 iterations x (2 Strong colours [+ RANSAC + 2 Weak])
    # + init + finish phases
    apd = bool(arr.params.use_APD)
    assert phases >= 1 + 3 * (2 + 3 * apd) + 4 + 3 * apd, phases
    assert accesses > arr.width * arr.height * 10
    assert n == 0, f"{n} conflicting accesses, first: {first}"
    ref = oracle_lib.run(oracle, arr, want_curve=True)
    diffs = cases.compare(ref, got)
    assert all(v == 0 for v in diffs.values()), diffs
    assert np.array_equal(ref.reliable_curve.view(np.uint32), got.reliable_curve.view(np.uint32))


@pytest.mark.parametrize("name", ["first_n4", "refine_iter_apd_geom_sa"])
def test_merged_colours_are_caught(name, oracle, rc):
    """Negative control: one launch over both colours of each checkerboard reads neighbours that
    the same launch writes (the propagation candidates are opposite-colour pixels)."""
    arr = cases.make_case(name, lambda a: oracle_lib.run(oracle, a))
    report(rc, merge_next=1)
    oracle_lib.run(rc, arr, nthreads=1)
    n, _, _, first = report(rc, merge_next=0)
    assert n > 0
    assert "run_iteration" in first or "run_finish" in first, first
