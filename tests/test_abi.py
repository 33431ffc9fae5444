"""C-ABI boundary checks that need no GPU: libapd_hip.so loads, exports every entry point declared in
include/*.h (apd_hip.h, apd_fusion.h), and the ctypes mirror has the exact C layout (compiled probe
with gcc)."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

import apd_abi as A

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "apd_hip.h")
HEADERS = [HEADER, os.path.join(REPO, "include", "apd_fusion.h")]


def declared_functions():
    src = "".join(open(h).read() for h in HEADERS)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(apd_[a-z_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    return A.load_library()


def test_every_declared_symbol_is_exported(lib):
    names = declared_functions()
    assert len(names) >= 22
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(A.EXPORTS)


def test_abi_version(lib):
    assert lib.apd_abi_version() == 3


def test_no_device_is_an_error_not_a_crash(lib):
    n = lib.apd_device_count()
    assert n >= 0
    if n == 0:
        assert not lib.apd_create(0)
        assert b"device" in lib.apd_last_error(None)
    assert not lib.apd_create(10_000)
    assert not lib.apd_fusion_create(10_000)
    assert b"device" in lib.apd_fusion_last_error(None)


def test_struct_layout_matches_header():
    probe = r'''
#include <stdio.h>
#include <stddef.h>
#include "apd_hip.h"
#include "apd_fusion.h"
#define P(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("apd_camera %zu\napd_params %zu\napd_problem %zu\napd_outputs %zu\napd_timing %zu\n",
         sizeof(apd_camera), sizeof(apd_params), sizeof(apd_problem), sizeof(apd_outputs), sizeof(apd_timing));
  P(apd_camera, depth_num) P(apd_params, state) P(apd_params, geom_factor) P(apd_problem, params)
  P(apd_problem, seed) P(apd_problem, sa_mask) P(apd_outputs, reliable_curve) P(apd_timing, iterations) P(apd_timing, pairs_ms)
  printf("apd_fusion_view %zu\n", sizeof(apd_fusion_view));
  P(apd_fusion_view, camera) P(apd_fusion_view, depth) P(apd_fusion_view, confidence)
  return 0;
}
'''
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "p.c")
        exe = os.path.join(d, "p")
        open(src, "w").write(probe)
        subprocess.run(["gcc", "-I", os.path.dirname(HEADER), "-o", exe, src], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split("\n")
    got = dict(l.rsplit(" ", 1) for l in out if l)
    assert int(got["apd_camera"]) == C.sizeof(A.ApdCamera) == 120  # Camera, main.h:50-61
    assert int(got["apd_params"]) == C.sizeof(A.ApdParams)
    assert int(got["apd_problem"]) == C.sizeof(A.ApdProblem)
    assert int(got["apd_outputs"]) == C.sizeof(A.ApdOutputs)
    assert int(got["apd_timing"]) == C.sizeof(A.ApdTiming)
    assert int(got["apd_camera.depth_num"]) == A.ApdCamera.depth_num.offset
    assert int(got["apd_params.state"]) == A.ApdParams.state.offset
    assert int(got["apd_params.geom_factor"]) == A.ApdParams.geom_factor.offset
    assert int(got["apd_problem.params"]) == A.ApdProblem.params.offset
    assert int(got["apd_problem.seed"]) == A.ApdProblem.seed.offset
    assert int(got["apd_problem.sa_mask"]) == A.ApdProblem.sa_mask.offset
    assert int(got["apd_outputs.reliable_curve"]) == A.ApdOutputs.reliable_curve.offset
    assert int(got["apd_timing.iterations"]) == A.ApdTiming.iterations.offset
    assert int(got["apd_timing.pairs_ms"]) == A.ApdTiming.pairs_ms.offset
    assert int(got["apd_fusion_view"]) == C.sizeof(A.ApdFusionView)
    assert int(got["apd_fusion_view.camera"]) == A.ApdFusionView.camera.offset
    assert int(got["apd_fusion_view.depth"]) == A.ApdFusionView.depth.offset
    assert int(got["apd_fusion_view.confidence"]) == A.ApdFusionView.confidence.offset


def test_epilogue_matches_process_problem(lib):
    """apd_epilogue == ProcessProblem's host loop (main.cpp:168-178)."""
    h, w = 5, 7
    rng = np.random.default_rng(0)
    planes = rng.uniform(-1, 12, (h, w, 4)).astype(np.float32)
    planes[0, 0, 3] = np.nan  # NaN depth passes the range test unchanged, as in the reference
    weak = np.full((h, w), A.STRONG, np.uint8)
    depth = np.zeros((h, w), np.float32)
    normal = np.zeros((h, w, 3), np.float32)
    st = lib.apd_epilogue(w, h, planes.ctypes.data_as(C.POINTER(C.c_float)), 1.0, 10.0,
                          depth.ctypes.data_as(C.POINTER(C.c_float)), normal.ctypes.data_as(C.POINTER(C.c_float)),
                          weak.ctypes.data_as(C.POINTER(C.c_uint8)))
    assert st == 0
    d = planes[..., 3]
    bad = (d < 1.0) | (d > 10.0)
    assert np.array_equal(weak, np.where(bad, A.UNKNOWN, A.STRONG).astype(np.uint8))
    assert np.array_equal(depth[~bad & ~np.isnan(d)], d[~bad & ~np.isnan(d)])
    assert (depth[bad] == 0).all() and np.isnan(depth[0, 0])
    assert np.array_equal(normal, planes[..., :3])
