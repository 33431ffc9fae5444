"""ctypes loader for the CPU parity oracle (oracle/liboracle.so). Test infrastructure only."""
import ctypes as C
import os
import subprocess

import numpy as np

import apd_abi as A

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")


ORACLE_FM_SO = os.path.join(ORACLE_DIR, "liboracle_fm.so")


def load(path=None):
    # APD_ORACLE_SO: a mutated oracle build (tools/mutate_oracle.py checks that the KATs reject it);
    # path=ORACLE_FM_SO: the fast-math variant of the numerics-sensitivity study (numerics_sensitivity.py)
    path = path or os.environ.get("APD_ORACLE_SO") or ORACLE_SO
    if path in (ORACLE_SO, ORACLE_FM_SO) and not os.path.exists(path):
        subprocess.run(["make", "-C", ORACLE_DIR, os.path.basename(path)], check=True, capture_output=True)
    lib = C.CDLL(path)
    lib.oracle_run_patchmatch.restype = C.c_int
    lib.oracle_run_patchmatch.argtypes = [C.POINTER(A.ApdProblem), C.POINTER(A.ApdOutputs), C.c_int,
                                          C.POINTER(C.c_double)]
    lib.oracle_time_iterations.restype = C.c_int
    lib.oracle_time_iterations.argtypes = [C.POINTER(A.ApdProblem), C.c_int, C.c_int, C.POINTER(C.c_double)]
    for name in ("oracle_ncc_old", "oracle_geom_cost"):
        f = getattr(lib, name)
        f.restype = C.c_float
        f.argtypes = [C.POINTER(A.ApdProblem), C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]
    lib.oracle_homography.restype = None
    lib.oracle_homography.argtypes = [C.POINTER(A.ApdProblem), C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float)]
    lib.oracle_depth_from_plane.restype = C.c_float
    lib.oracle_depth_from_plane.argtypes = [C.POINTER(A.ApdCamera), C.POINTER(C.c_float), C.c_int, C.c_int]
    lib.oracle_dist2origin.restype = C.c_float
    lib.oracle_dist2origin.argtypes = [C.POINTER(A.ApdCamera), C.c_int, C.c_int, C.c_float, C.POINTER(C.c_float)]
    lib.oracle_tex_bilinear.restype = C.c_float
    lib.oracle_tex_bilinear.argtypes = [C.POINTER(C.c_float), C.c_int, C.c_int, C.c_float, C.c_float]
    for name in ("oracle_expf", "oracle_sinf", "oracle_cosf"):
        f = getattr(lib, name)
        f.restype = C.c_float
        f.argtypes = [C.c_float]
    lib.oracle_philox.restype = None
    lib.oracle_philox.argtypes = [C.POINTER(C.c_uint32), C.c_uint32, C.c_uint32]
    return lib


def run(lib, arrays: "A.ProblemArrays", nthreads: int = 0, want_curve: bool = False):
    pb = arrays.build()
    n_src = len(arrays.images) - 1
    hw = arrays.width * arrays.height
    out = A.Outputs(arrays.width, arrays.height, n_src, want_curve=want_curve, max_weak=hw)
    times = (C.c_double * 3)()
    st = lib.oracle_run_patchmatch(C.byref(pb), C.byref(out.struct()), nthreads, times)
    if st != 0:
        raise RuntimeError(f"oracle_run_patchmatch -> {st}")
    out.times = list(times)
    return out


def f4(v):
    a = np.asarray(v, np.float32)
    return a.ctypes.data_as(C.POINTER(C.c_float)), a
