"""ctypes mirror of include/apd_hip.h and a thin Python driver for libapd_hip.so.

This is plumbing for tests and bench.py: the product is the C-ABI library itself. The structures
below are byte-for-byte the C ones; `ProblemArrays` keeps the numpy buffers alive while a call is in
flight. Loading fails loudly (ApdError) when the HIP library is missing: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB_PATH = os.environ.get("APD_LIB") or os.path.join(HERE, "lib", "libapd_hip.so")  # APD_LIB: A/B tooling

MAX_IMAGES = 32
ANCHOR_NUM = 9
FIRST_INIT, REFINE_INIT, REFINE_ITER = 0, 1, 2
WEAK, STRONG, UNKNOWN = 0, 1, 2

# apd_profile_kernel kinds and apd_profile_counters slots (include/apd_hip.h)
PROF_STRONG_SWEEP, PROF_RANSAC_FIT, PROF_WEAK_CAND, PROF_WEAK_SWEEP = 0, 1, 2, 3
PROF_DEPTH_TO_WEAK, PROF_GP_COST, PROF_WEAK_CAND_G, PROF_WEAK_CAND_COMB, PROF_WEAK_PATH = 4, 5, 6, 7, 8
# apd_hip.h's counters: [0] NCC-Old (Strong sweep), [1] NCC-New (Weak sweep, algorithmic), [2] geometric
# terms (Weak sweep), [3] NCC-Old (DepthToWeak), [4] geometric terms (DepthToWeak), [5] pair windows
# (k_gp_cost), [6] centre windows (k_weak_cand_g), [7] centre / [8] anchor windows (k_sweep_weak_vm)
PROF_COUNTERS = 9

STATUS = {0: "APD_OK", -1: "APD_EINVAL", -2: "APD_ENOMEM", -3: "APD_EDEVICE", -4: "APD_ETOOMANYVIEWS",
          -5: "APD_ESTATE"}


class ApdError(RuntimeError):
    pass


class ApdCamera(C.Structure):
    _fields_ = [("K", C.c_float * 9), ("R", C.c_float * 9), ("t", C.c_float * 3), ("c", C.c_float * 3),
                ("height", C.c_int32), ("width", C.c_int32), ("depth_min", C.c_float), ("depth_max", C.c_float),
                ("interval", C.c_float), ("depth_num", C.c_float)]


assert C.sizeof(ApdCamera) == 120


class ApdParams(C.Structure):
    _fields_ = [("max_iterations", C.c_int32), ("num_images", C.c_int32), ("top_k", C.c_int32),
                ("depth_min", C.c_float), ("depth_max", C.c_float), ("geom_consistency", C.c_int32),
                ("use_impetus", C.c_int32), ("strong_radius", C.c_int32), ("strong_increment", C.c_int32),
                ("weak_radius", C.c_int32), ("weak_increment", C.c_int32), ("use_APD", C.c_int32),
                ("use_sa", C.c_int32), ("weak_peak_radius", C.c_int32), ("rotate_time", C.c_int32),
                ("ransac_threshold", C.c_float), ("geom_factor", C.c_float), ("state", C.c_int32)]


class ApdProblem(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("num_images", C.c_int32),
                ("images", C.POINTER(C.POINTER(C.c_float))), ("cameras", C.POINTER(ApdCamera)),
                ("params", ApdParams), ("depths", C.POINTER(C.POINTER(C.c_float))),
                ("init_planes", C.POINTER(C.c_float)), ("weak_info", C.POINTER(C.c_uint8)),
                ("confidence", C.POINTER(C.c_uint8)), ("sa_mask", C.POINTER(C.c_uint8)), ("seed", C.c_uint64),
                ("export_reliable_curve", C.c_int32)]


class ApdOutputs(C.Structure):
    _fields_ = [("planes", C.POINTER(C.c_float)), ("weak_info", C.POINTER(C.c_uint8)),
                ("confidence", C.POINTER(C.c_uint8)), ("costs", C.POINTER(C.c_float)),
                ("selected_views", C.POINTER(C.c_uint32)), ("view_weights", C.POINTER(C.c_uint8)),
                ("anchors", C.POINTER(C.c_int16)), ("weak_count", C.POINTER(C.c_int32)),
                ("reliable_curve", C.POINTER(C.c_float))]


class ApdTiming(C.Structure):
    _fields_ = [("total_ms", C.c_float), ("init_ms", C.c_float), ("anchors_ms", C.c_float),
                ("sweep_ms", C.c_float), ("post_ms", C.c_float), ("iter_ms", C.c_float * 8),
                ("iterations", C.c_int32), ("lists_ms", C.c_float), ("pairs_ms", C.c_float),
                ("join_ms", C.c_float), ("prepare_ms", C.c_float)]


def default_params(num_images: int, depth_min: float, depth_max: float, **kw) -> ApdParams:
    """PatchMatchParams defaults (main.h:80-100) with the scaled depth range (APD.cpp:554-555)."""
    p = ApdParams(max_iterations=3, num_images=num_images, top_k=4, depth_min=depth_min, depth_max=depth_max,
                  geom_consistency=0, use_impetus=1, strong_radius=5, strong_increment=2, weak_radius=5,
                  weak_increment=5, use_APD=0, use_sa=1, weak_peak_radius=6, rotate_time=4,
                  ransac_threshold=0.005, geom_factor=0.2, state=FIRST_INIT)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _ptr(a, ctype):
    """ctypes pointer to a numpy array's or a torch tensor's data (host or device memory: the C ABI
    accepts device pointers for the problem arrays and the outputs)."""
    if a is None:
        return C.POINTER(ctype)()
    if hasattr(a, "data_ptr"):
        return C.cast(C.c_void_p(a.data_ptr()), C.POINTER(ctype))
    return a.ctypes.data_as(C.POINTER(ctype))


_TORCH_DTYPES = {np.dtype(np.float32): "float32", np.dtype(np.uint8): "uint8"}


def _torch_device_sync(*objs):
    """Wait for torch's current stream on the device of every CUDA tensor in `objs` (lists/tuples
    are searched one level deep). The library works on its own non-blocking HIP stream, which does
    not wait for torch's stream or for RCCL's: a tensor torch (an index_select, a .to(), a cat, an
    all_gather) has just produced may still be in flight when the library reads it, and a fresh
    torch.empty may reuse memory a pending torch kernel still touches."""
    seen = set()
    for o in objs:
        for t in (o if isinstance(o, (list, tuple)) else (o,)):
            if t is None or not hasattr(t, "is_cuda") or not t.is_cuda:
                continue
            if t.device.index in seen:
                continue
            seen.add(t.device.index)
            import torch
            torch.cuda.current_stream(t.device).synchronize()


def _keep(a, dtype):
    """A contiguous buffer of `dtype` holding `a` (numpy array or torch tensor, kept as a tensor)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        import torch
        t = a.contiguous()
        want = getattr(torch, _TORCH_DTYPES[np.dtype(dtype)])
        return t if t.dtype == want else t.to(want)
    return np.ascontiguousarray(a, dtype)


@dataclass
class ProblemArrays:
    """Owns every numpy buffer an ApdProblem points into."""
    width: int
    height: int
    images: Sequence[np.ndarray]
    cameras: Sequence[dict]
    params: ApdParams
    depths: Optional[Sequence[np.ndarray]] = None
    init_planes: Optional[np.ndarray] = None  # HxWx4 {world normal, depth}
    weak_info: Optional[np.ndarray] = None
    confidence: Optional[np.ndarray] = None
    sa_mask: Optional[np.ndarray] = None
    seed: int = 0x5EED
    export_reliable_curve: bool = False

    def build(self) -> ApdProblem:
        n = len(self.images)
        self._imgs = [_keep(i, np.float32) for i in self.images]
        self._img_ptrs = (C.POINTER(C.c_float) * n)(*[_ptr(i, C.c_float) for i in self._imgs])
        self._cams = (ApdCamera * n)()
        for i, cv in enumerate(self.cameras):
            cam = self._cams[i]
            for k, v in cv.items():
                if isinstance(v, np.ndarray):
                    getattr(cam, k)[:] = [float(x) for x in v]
                else:
                    setattr(cam, k, v)
        if self.depths is not None:
            self._deps = [_keep(d, np.float32) for d in self.depths]
            dptrs = (C.POINTER(C.c_float) * n)(*[_ptr(d, C.c_float) for d in self._deps])
            self._dep_ptrs = dptrs
        else:
            self._dep_ptrs = None
        self._planes = _keep(self.init_planes, np.float32)
        self._weak = _keep(self.weak_info, np.uint8)
        self._conf = _keep(self.confidence, np.uint8)
        self._sa = _keep(self.sa_mask, np.uint8)
        pb = ApdProblem()
        pb.width, pb.height, pb.num_images = self.width, self.height, n
        pb.images = C.cast(self._img_ptrs, C.POINTER(C.POINTER(C.c_float)))
        pb.cameras = C.cast(self._cams, C.POINTER(ApdCamera))
        pb.params = self.params
        pb.params.num_images = n
        pb.depths = C.cast(self._dep_ptrs, C.POINTER(C.POINTER(C.c_float))) if self._dep_ptrs is not None \
            else C.POINTER(C.POINTER(C.c_float))()
        pb.init_planes = _ptr(self._planes, C.c_float)
        pb.weak_info = _ptr(self._weak, C.c_uint8)
        pb.confidence = _ptr(self._conf, C.c_uint8)
        pb.sa_mask = _ptr(self._sa, C.c_uint8)
        pb.seed = self.seed
        pb.export_reliable_curve = int(self.export_reliable_curve)
        self._pb = pb
        return pb


class Outputs:
    """Host buffers for apd_outputs, allocated for one problem size."""

    def __init__(self, width: int, height: int, num_src: int, want_curve: bool = False, max_weak: int = 0):
        hw = width * height
        self.planes = np.zeros((height, width, 4), np.float32)
        self.weak_info = np.zeros((height, width), np.uint8)
        self.confidence = np.zeros((height, width), np.uint8)
        self.costs = np.zeros((height, width), np.float32)
        self.selected_views = np.zeros((height, width), np.uint32)
        self.view_weights = np.zeros((num_src, height, width), np.uint8)
        # anchors are only requested when the caller sizes them (weak_count <= max_weak): the library
        # writes weak_count * 9 entries, so an undersized buffer must never be handed over
        self.anchors = np.zeros((max_weak, ANCHOR_NUM, 2), np.int16) if max_weak > 0 else None
        self.weak_count = np.zeros(1, np.int32)
        self.reliable_curve = np.zeros((hw, 61), np.float32) if want_curve else None

    def struct(self) -> ApdOutputs:
        o = ApdOutputs()
        o.planes = _ptr(self.planes, C.c_float)
        o.weak_info = _ptr(self.weak_info, C.c_uint8)
        o.confidence = _ptr(self.confidence, C.c_uint8)
        o.costs = _ptr(self.costs, C.c_float)
        o.selected_views = _ptr(self.selected_views, C.c_uint32)
        o.view_weights = _ptr(self.view_weights, C.c_uint8)
        o.anchors = _ptr(self.anchors, C.c_int16)  # NULL when not sized
        o.weak_count = _ptr(self.weak_count, C.c_int32)
        o.reliable_curve = _ptr(self.reliable_curve, C.c_float)
        return o


EXPORTS = ["apd_abi_version", "apd_device_count", "apd_create", "apd_destroy", "apd_last_error",
           "apd_set_problem", "apd_run_patchmatch", "apd_stage_prepare", "apd_stage_iteration",
           "apd_stage_finish", "apd_synchronize", "apd_get_results", "apd_get_timing", "apd_get_prepare_timing", "apd_profile_reset",
           "apd_profile_query", "apd_profile_kernel", "apd_profile_counters", "apd_profile_evaluations", "apd_epilogue", "apd_device_alloc", "apd_device_free",
           "apd_device_copy", "apd_device_copy_peer", "apd_device_bytes", "apd_device_mem_info", "apd_device_resize_nearest", "apd_result_device", "apd_fusion_create", "apd_fusion_destroy",
           "apd_fusion_last_error", "apd_fusion_set_views", "apd_fusion_weak_filter", "apd_fusion_consistency",
           "apd_fusion_tat_levels"]


class ApdFusionView(C.Structure):  # include/apd_fusion.h
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("camera", ApdCamera),
                ("depth", C.c_void_p), ("normal", C.c_void_p), ("weak", C.c_void_p), ("confidence", C.c_void_p)]


def torch_runtime_first():
    """One HIP runtime per process. torch ships its own libamdhip64 (soname libamdhip64.so.7) and its
    libraries load it by the file name libamdhip64.so: loaded after ours (/opt/rocm's, the same
    soname) it would be a second runtime, which finds no GPU. Loaded first, it satisfies our
    dependency too, so torch tensors and this library share one runtime (device pointers pass
    through the C ABI). Call before loading anything that links libapd_hip.so; without torch the
    library uses /opt/rocm's runtime."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load_library(path: str = LIB_PATH) -> C.CDLL:
    if not os.path.exists(path):
        raise ApdError(f"libapd_hip.so not built at {path}: run `python -c 'import __graft_entry__ as g; g.build()'`")
    torch_runtime_first()
    lib = C.CDLL(path)
    lib.apd_abi_version.restype = C.c_int32
    lib.apd_device_count.restype = C.c_int32
    lib.apd_create.restype = C.c_void_p
    lib.apd_create.argtypes = [C.c_int32]
    lib.apd_destroy.argtypes = [C.c_void_p]
    lib.apd_last_error.restype = C.c_char_p
    lib.apd_last_error.argtypes = [C.c_void_p]
    for name in ["apd_run_patchmatch", "apd_stage_prepare", "apd_stage_finish", "apd_synchronize"]:
        getattr(lib, name).restype = C.c_int32
        getattr(lib, name).argtypes = [C.c_void_p]
    lib.apd_set_problem.restype = C.c_int32
    lib.apd_set_problem.argtypes = [C.c_void_p, C.POINTER(ApdProblem)]
    lib.apd_stage_iteration.restype = C.c_int32
    lib.apd_stage_iteration.argtypes = [C.c_void_p, C.c_int32]
    lib.apd_get_results.restype = C.c_int32
    lib.apd_get_results.argtypes = [C.c_void_p, C.POINTER(ApdOutputs)]
    lib.apd_get_timing.restype = C.c_int32
    lib.apd_get_timing.argtypes = [C.c_void_p, C.POINTER(ApdTiming)]
    lib.apd_get_prepare_timing.restype = C.c_int32
    lib.apd_get_prepare_timing.argtypes = [C.c_void_p, C.POINTER(ApdTiming)]
    lib.apd_profile_reset.restype = C.c_int32
    lib.apd_profile_reset.argtypes = [C.c_void_p, C.c_int32]
    lib.apd_profile_evaluations.restype = C.c_int32
    lib.apd_profile_evaluations.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
    lib.apd_profile_query.restype = C.c_int32
    lib.apd_profile_query.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int64),
                                      C.POINTER(C.c_int64)]
    lib.apd_profile_kernel.restype = C.c_int32
    lib.apd_profile_kernel.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_int64),
                                       C.POINTER(C.c_int64)]
    lib.apd_profile_counters.restype = C.c_int32
    lib.apd_profile_counters.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.c_int32]
    lib.apd_device_alloc.restype = C.c_int32
    lib.apd_device_alloc.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]
    lib.apd_device_free.restype = C.c_int32
    lib.apd_device_free.argtypes = [C.c_void_p, C.c_void_p]
    lib.apd_device_copy.restype = C.c_int32
    lib.apd_device_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
    lib.apd_device_mem_info.restype = C.c_int32
    lib.apd_device_mem_info.argtypes = [C.c_void_p, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
    lib.apd_device_resize_nearest.restype = C.c_int32
    lib.apd_device_resize_nearest.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32,
                                              C.c_int32, C.c_int32]
    lib.apd_result_device.restype = C.c_int32
    lib.apd_result_device.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.apd_fusion_create.restype = C.c_void_p
    lib.apd_fusion_create.argtypes = [C.c_int32]
    lib.apd_fusion_destroy.argtypes = [C.c_void_p]
    lib.apd_fusion_last_error.restype = C.c_char_p
    lib.apd_fusion_last_error.argtypes = [C.c_void_p]
    lib.apd_fusion_set_views.restype = C.c_int32
    lib.apd_fusion_set_views.argtypes = [C.c_void_p, C.c_int32, C.POINTER(ApdFusionView)]
    lib.apd_fusion_weak_filter.restype = C.c_int32
    lib.apd_fusion_weak_filter.argtypes = [C.c_void_p, C.c_int32, C.c_float, C.c_void_p]
    lib.apd_fusion_consistency.restype = C.c_int32
    lib.apd_fusion_consistency.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_float, C.c_void_p,
                                           C.c_void_p, C.c_void_p]
    lib.apd_fusion_tat_levels.restype = C.c_int32
    lib.apd_fusion_tat_levels.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_float, C.c_float,
                                          C.c_void_p, C.c_void_p, C.c_void_p]
    lib.apd_epilogue.restype = C.c_int32
    lib.apd_epilogue.argtypes = [C.c_int32, C.c_int32, C.POINTER(C.c_float), C.c_float, C.c_float,
                                 C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_uint8)]
    return lib


class FusionEngine:
    """One apd_fusion_ctx (include/apd_fusion.h) with its views resident on the device."""

    def __init__(self, device: int = 0, lib: Optional[C.CDLL] = None):
        self.lib = lib or load_library()
        self.ctx = self.lib.apd_fusion_create(device)
        if not self.ctx:
            raise ApdError("apd_fusion_create failed: " + (self.lib.apd_fusion_last_error(None) or b"?").decode())

    def _check(self, st: int, what: str):
        if st != 0:
            msg = (self.lib.apd_fusion_last_error(self.ctx) or b"").decode()
            raise ApdError(f"{what} -> {STATUS.get(st, st)}: {msg}")

    def set_views(self, views):
        """views: dicts with depth (H,W) f32, normal (H,W,3) f32, weak/conf (H,W) u8, cam ApdCamera."""
        self._views = views
        arr = (ApdFusionView * len(views))()
        for i, v in enumerate(views):
            arr[i] = ApdFusionView(v["depth"].shape[1], v["depth"].shape[0], v["cam"], v["depth"].ctypes.data,
                                   v["normal"].ctypes.data, v["weak"].ctypes.data, v["conf"].ctypes.data)
        self._check(self.lib.apd_fusion_set_views(self.ctx, len(views), arr), "apd_fusion_set_views")

    def weak_filter(self, ref: int, q_view: float) -> np.ndarray:
        out = np.zeros(self._views[ref]["depth"].shape, np.uint8)
        self._check(self.lib.apd_fusion_weak_filter(self.ctx, ref, q_view, out.ctypes.data), "apd_fusion_weak_filter")
        return out

    def consistency(self, ref: int, src: Sequence[int], q_angle: float):
        H, W = self._views[ref]["depth"].shape
        s = np.asarray(src, np.int32)
        pix = np.zeros((H, W, len(s)), np.int32)
        er = np.zeros((H, W, len(s)), np.float32)
        q = np.zeros((H, W, len(s)), np.float32)
        self._check(self.lib.apd_fusion_consistency(self.ctx, ref, len(s), s.ctypes.data, q_angle, pix.ctypes.data,
                                                    er.ctypes.data, q.ctypes.data), "apd_fusion_consistency")
        return pix, er, q

    def tat_levels(self, ref: int, src: Sequence[int], dist_base: float, depth_base: float, q_k=None):
        H, W = self._views[ref]["depth"].shape
        s = np.asarray(src, np.int32)
        pix = np.zeros((H, W, len(s)), np.int32)
        lv = np.zeros((H, W, len(s)), np.uint8)
        qk = None if q_k is None else np.asarray(q_k, np.float32)
        self._check(self.lib.apd_fusion_tat_levels(self.ctx, ref, len(s), s.ctypes.data, dist_base, depth_base,
                                                   None if qk is None else qk.ctypes.data, pix.ctypes.data,
                                                   lv.ctypes.data), "apd_fusion_tat_levels")
        return pix, lv

    def close(self):
        if self.ctx:
            self.lib.apd_fusion_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Engine:
    """One apd_ctx on one HIP device."""

    def __init__(self, device: int = 0, lib: Optional[C.CDLL] = None):
        self.lib = lib or load_library()
        self.ctx = self.lib.apd_create(device)
        if not self.ctx:
            raise ApdError("apd_create failed: " + (self.lib.apd_last_error(None) or b"?").decode())

    def _check(self, st: int, what: str):
        if st != 0:
            msg = (self.lib.apd_last_error(self.ctx) or b"").decode()
            raise ApdError(f"{what} -> {STATUS.get(st, st)}: {msg}")

    def set_problem(self, arrays: ProblemArrays):
        pb = arrays.build()
        self._arrays = arrays
        # device-resident inputs (scan_runner.py) may be fresh outputs of torch / RCCL kernels
        _torch_device_sync(arrays._imgs, getattr(arrays, "_deps", None), arrays._planes, arrays._weak,
                           arrays._conf, arrays._sa)
        self._check(self.lib.apd_set_problem(self.ctx, C.byref(pb)), "apd_set_problem")

    def run(self):
        self._check(self.lib.apd_run_patchmatch(self.ctx), "apd_run_patchmatch")

    def prepare(self):
        self._check(self.lib.apd_stage_prepare(self.ctx), "apd_stage_prepare")

    def iteration(self, i: int):
        self._check(self.lib.apd_stage_iteration(self.ctx, i), "apd_stage_iteration")

    def finish(self):
        self._check(self.lib.apd_stage_finish(self.ctx), "apd_stage_finish")

    def synchronize(self):
        self._check(self.lib.apd_synchronize(self.ctx), "apd_synchronize")

    def results(self, out: Outputs):
        s = out.struct()
        self._check(self.lib.apd_get_results(self.ctx, C.byref(s)), "apd_get_results")
        return out

    def results_device(self, width: int, height: int, device: str):
        """planes / weak_info / confidence as torch tensors on `device` (the ctx's device), copied
        device to device by apd_get_results."""
        import torch
        from types import SimpleNamespace
        o = SimpleNamespace(planes=torch.empty((height, width, 4), dtype=torch.float32, device=device),
                            weak_info=torch.empty((height, width), dtype=torch.uint8, device=device),
                            confidence=torch.empty((height, width), dtype=torch.uint8, device=device))
        s = ApdOutputs()
        s.planes = _ptr(o.planes, C.c_float)
        s.weak_info = _ptr(o.weak_info, C.c_uint8)
        s.confidence = _ptr(o.confidence, C.c_uint8)
        _torch_device_sync(o.planes)
        self._check(self.lib.apd_get_results(self.ctx, C.byref(s)), "apd_get_results")
        return o

    def resize_nearest_device(self, src, dw: int, dh: int):
        """apd_device_resize_nearest of a contiguous (H, W[, C]) torch tensor on the ctx's device."""
        import torch
        src = src.contiguous()
        sh, sw = src.shape[:2]
        dst = torch.empty((dh, dw) + tuple(src.shape[2:]), dtype=src.dtype, device=src.device)
        elem = src.element_size() * (src[0, 0].numel() if src.dim() > 2 else 1)
        _torch_device_sync(src, dst)
        self._check(self.lib.apd_device_resize_nearest(self.ctx, src.data_ptr(), sw, sh, dst.data_ptr(), dw, dh, elem),
                    "apd_device_resize_nearest")
        return dst

    def result_device(self, width: int, height: int, device: str):
        """apd_result_device: (depth (H, W), planes (H, W, 4)) of the last run, epilogue applied, on `device`."""
        import torch
        depth = torch.empty((height, width), dtype=torch.float32, device=device)
        planes = torch.empty((height, width, 4), dtype=torch.float32, device=device)
        _torch_device_sync(depth, planes)
        self._check(self.lib.apd_result_device(self.ctx, depth.data_ptr(), planes.data_ptr()), "apd_result_device")
        return depth, planes

    def timing(self) -> ApdTiming:
        t = ApdTiming()
        self._check(self.lib.apd_get_timing(self.ctx, C.byref(t)), "apd_get_timing")
        return t

    def prepare_timing(self) -> ApdTiming:
        """The prepare-phase fields of the last apd_stage_prepare (waits for the ctx stream)."""
        t = ApdTiming()
        self._check(self.lib.apd_get_prepare_timing(self.ctx, C.byref(t)), "apd_get_prepare_timing")
        return t

    def profile_reset(self, enable: bool = True):
        self._check(self.lib.apd_profile_reset(self.ctx, int(enable)), "apd_profile_reset")

    def profile_query(self):
        ms, n, px = C.c_double(), C.c_int64(), C.c_int64()
        self._check(self.lib.apd_profile_query(self.ctx, C.byref(ms), C.byref(n), C.byref(px)), "apd_profile_query")
        return ms.value, n.value, px.value

    def profile_kernel(self, kind: int):
        """(total ms, launches, pixels) of the profiled launches of one APD_PROF_* kind."""
        ms, n, px = C.c_double(), C.c_int64(), C.c_int64()
        self._check(self.lib.apd_profile_kernel(self.ctx, kind, C.byref(ms), C.byref(n), C.byref(px)),
                    "apd_profile_kernel")
        return ms.value, n.value, px.value

    def profile_counters(self):
        c = (C.c_int64 * PROF_COUNTERS)()
        self._check(self.lib.apd_profile_counters(self.ctx, c, PROF_COUNTERS), "apd_profile_counters")
        return list(c)

    def profile_evaluations(self) -> int:
        n = C.c_int64()
        self._check(self.lib.apd_profile_evaluations(self.ctx, C.byref(n)), "apd_profile_evaluations")
        return n.value

    def close(self):
        if self.ctx:
            self.lib.apd_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def scene_problem(scene, ref: int = 0, srcs: Optional[Sequence[int]] = None, params: Optional[ApdParams] = None,
                  seed: int = 0x5EED, **kw) -> ProblemArrays:
    """ProblemArrays for one reference view of a synth.Scene (full resolution, FIRST_INIT defaults)."""
    from importlib import import_module
    synth = import_module("synth")
    if srcs is None:
        srcs = [j for j, _ in scene.pairs[ref]]
    ids = [ref] + list(srcs)
    cams = [synth.camera_struct_values(scene.cameras[i], scene.width, scene.height) for i in ids]
    c0 = scene.cameras[ref]
    if params is None:
        params = default_params(len(ids), float(np.float32(c0.depth_min) * np.float32(0.6)),
                                float(np.float32(c0.depth_max) * np.float32(1.2)))
    return ProblemArrays(scene.width, scene.height, [scene.images[i] for i in ids], cams, params, seed=seed, **kw)
