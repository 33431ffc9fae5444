"""Fusion test helpers: synthetic fused-scan folders, the C oracle (oracle/fusion_oracle.c) through
ctypes, the host helpers of libapdhost.so, and a PLY reader.

A fusion scan is an MVSNet folder (images/, cams/, pair.txt) plus the depth stage's outputs under
APD/<id>/ (depths.bin, normals.bin, weak.bin, confidence.bin) -- exactly what RunFusion reads
(APD.cpp:1071-1133). Depths are the synthetic scene's ground truth with multiplicative noise, holes
and negative values; normals are the scene planes' normals in each camera frame with noise (and a
few zero vectors, which make GetAngle's acosf NaN); weak/confidence are random with flat regions.
"""
import ctypes as C
import os
import subprocess

import numpy as np
from PIL import Image

import apd_abi as A
import synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle.so")
HOST_SO = os.path.join(REPO, "apde-mvs_amd", "host", "build", "libapdhost.so")
APD_BIN = os.path.join(REPO, "apde-mvs_amd", "host", "build", "apd")


class OracleFusionView(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("camera", A.ApdCamera),
                ("depth", C.c_void_p), ("normal", C.c_void_p), ("weak", C.c_void_p),
                ("confidence", C.c_void_p), ("bgr", C.c_void_p), ("ref_id", C.c_int32),
                ("num_src", C.c_int32), ("src_ids", C.c_void_p)]


def oracle():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", os.path.dirname(ORACLE_SO)], check=True, capture_output=True)
    lib = C.CDLL(ORACLE_SO)
    lib.oracle_fusion.restype = C.c_int64
    lib.oracle_fusion.argtypes = [C.c_int, C.c_int, C.POINTER(OracleFusionView), C.c_int,
                                  C.POINTER(C.c_void_p), C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    return lib


def hostlib():
    A.torch_runtime_first()  # libapdhost.so links libapd_hip.so
    lib = C.CDLL(HOST_SO)
    lib.apdhost_read_bgr8.restype = C.c_long
    lib.apdhost_read_bgr8.argtypes = [C.c_char_p, C.c_void_p, C.c_long, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    lib.apdhost_resize_linear_u8c3.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int]
    lib.apdhost_write_png_gray8.argtypes = [C.c_char_p, C.c_void_p, C.c_int, C.c_int]
    lib.apdhost_angle_cut_lt.restype = C.c_float
    lib.apdhost_angle_cut_lt.argtypes = [C.c_float]
    lib.apdhost_view_cut_deg.restype = C.c_float
    lib.apdhost_view_cut_deg.argtypes = [C.c_float]
    lib.apdhost_read_camera.argtypes = [C.c_char_p, C.POINTER(A.ApdCamera)]
    return lib


def read_bgr(lib, path):
    w, h = C.c_int(), C.c_int()
    n = lib.apdhost_read_bgr8(path.encode(), None, 0, C.byref(w), C.byref(h))
    assert n > 0, f"cannot decode {path}"
    out = np.empty(n, np.uint8)
    lib.apdhost_read_bgr8(path.encode(), out.ctypes.data, n, C.byref(w), C.byref(h))
    return out.reshape(h.value, w.value, 3)


def resize_bgr(lib, img, w, h):
    src = np.ascontiguousarray(img, np.uint8)
    dst = np.empty((h, w, 3), np.uint8)
    lib.apdhost_resize_linear_u8c3(src.ctypes.data, src.shape[1], src.shape[0], dst.ctypes.data, w, h)
    return dst


def make_fusion_scan(folder, width=96, height=72, n_src=4, seed=11, image_scale=1, noise=0.0003):
    """Writes a fusion-ready scan; returns the scene. image_scale > 1 stores colour images larger
    than the depth maps (RescaleImageAndCamera path)."""
    sc = synth.make_scene(width, height, n_src, seed=seed)
    rng = np.random.default_rng(seed + 1)
    os.makedirs(os.path.join(folder, "images"), exist_ok=True)
    os.makedirs(os.path.join(folder, "cams"), exist_ok=True)
    nv = len(sc.images)
    iw, ih = int(round(width * image_scale)), int(round(height * image_scale))
    for i, cam in enumerate(sc.cameras):
        name = f"{i:08d}"
        g = sc.images[i].astype(np.float64)
        rgb = np.stack([g, 255 - g, rng.integers(0, 256, g.shape)], -1).astype(np.uint8)
        img = Image.fromarray(rgb, "RGB")
        if (iw, ih) != (width, height):
            img = img.resize((iw, ih), Image.NEAREST)
        img.save(os.path.join(folder, "images", name + ".png"))
        K = cam.K.copy()
        K[0] *= iw / width
        K[1] *= ih / height
        with open(os.path.join(folder, "cams", name + "_cam.txt"), "w") as fh:
            fh.write("extrinsic\n")
            for r in range(3):
                fh.write(" ".join(repr(float(v)) for v in cam.R[r]) + " " + repr(float(cam.t[r])) + "\n")
            fh.write("0.0 0.0 0.0 1.0\n\nintrinsic\n")
            for r in range(3):
                fh.write(" ".join(repr(float(v)) for v in K[r]) + "\n")
            fh.write(f"\n{cam.depth_min!r} {cam.interval!r} {cam.depth_num!r} {cam.depth_max!r}\n")
    with open(os.path.join(folder, "pair.txt"), "w") as fh:
        fh.write(f"{nv}\n")
        for i, pl in enumerate(sc.pairs):
            fh.write(f"{i}\n{len(pl)} " + " ".join(f"{j} {s}" for j, s in pl) + "\n")
    for i in range(nv):
        d = os.path.join(folder, "APD", f"{i:08d}")
        os.makedirs(d, exist_ok=True)
        gt = sc.gt_depth[i]
        depth = (gt * (1.0 + rng.normal(0.0, noise, gt.shape))).astype(np.float32)
        depth[rng.random(gt.shape) < 0.08] *= 1.25  # outliers behind the surface: WeakVisFilter occlusions
        depth[rng.random(gt.shape) < 0.03] = 0.0
        depth[rng.random(gt.shape) < 0.01] = -1.0
        # camera-frame surface normals of the GT geometry (cross product of the back-projected
        # neighbours), so the same surface has nearly the same normal in every view
        Kinv = np.linalg.inv(cam_k(sc.cameras[i]))
        ys, xs = np.mgrid[0:height, 0:width].astype(np.float64)
        rays = np.stack([xs, ys, np.ones_like(xs)], -1) @ Kinv.T
        P = rays * gt[..., None].astype(np.float64)
        du = np.gradient(P, axis=1)
        dv = np.gradient(P, axis=0)
        n = np.cross(du, dv)
        n /= np.maximum(np.linalg.norm(n, axis=-1, keepdims=True), 1e-12)
        n = np.where((n[..., 2:3] > 0), -n, n)  # face the camera
        n += rng.normal(0.0, 0.01, n.shape)
        n = n.astype(np.float32)
        n[rng.random(gt.shape) < 0.005] = 0.0
        weak = rng.choice(np.array([0, 1, 2], np.uint8), size=gt.shape, p=[0.35, 0.6, 0.05])
        weak[: height // 3, : width // 2] = 0  # a WEAK block (WeakVisFilter work)
        conf = rng.integers(0, 256, gt.shape).astype(np.uint8)
        synth.write_bin_mat(os.path.join(d, "depths.bin"), depth)
        synth.write_bin_mat(os.path.join(d, "normals.bin"), n)
        synth.write_bin_mat(os.path.join(d, "weak.bin"), weak)
        synth.write_bin_mat(os.path.join(d, "confidence.bin"), conf)
    return sc


def cam_k(cam):
    return cam.K


def load_views(folder, hl):
    """What RunFusion loads (APD.cpp:1071-1133), read with the host helpers (decode, cam parsing) and
    rescaled like RescaleImageAndCamera (APD.cpp:844-864)."""
    with open(os.path.join(folder, "pair.txt")) as fh:
        lines = fh.read().split("\n")
    nv = int(lines[0])
    views = []
    for i in range(nv):
        ref = int(lines[1 + 2 * i])
        toks = lines[2 + 2 * i].split()
        srcs = [int(toks[1 + 2 * k]) for k in range(int(toks[0])) if float(toks[2 + 2 * k]) > 0]
        name = f"{ref:08d}"
        d = os.path.join(folder, "APD", name)
        depth = synth.read_bin_mat(os.path.join(d, "depths.bin"))
        H, W = depth.shape
        cam = A.ApdCamera()
        assert hl.apdhost_read_camera(os.path.join(folder, "cams", name + "_cam.txt").encode(), C.byref(cam)) == 0
        bgr = read_bgr(hl, os.path.join(folder, "images", name + ".png"))
        if bgr.shape[:2] != (H, W):
            sx = np.float32(W) / np.float32(bgr.shape[1])
            sy = np.float32(H) / np.float32(bgr.shape[0])
            bgr = resize_bgr(hl, bgr, W, H)
            for k, s in ((0, sx), (2, sx), (4, sy), (5, sy)):
                cam.K[k] = float(np.float32(cam.K[k]) * s)
            cam.width, cam.height = W, H
        views.append(dict(ref=ref, srcs=srcs, depth=depth,
                          normal=synth.read_bin_mat(os.path.join(d, "normals.bin")),
                          weak=synth.read_bin_mat(os.path.join(d, "weak.bin")),
                          conf=synth.read_bin_mat(os.path.join(d, "confidence.bin")),
                          bgr=np.ascontiguousarray(bgr), cam=cam))
    return views


VARIANTS = {"ETH3D": 0, "TaT_i": 1, "TaT_a": 2}


def _oracle_views(views):
    n = len(views)
    arr = (OracleFusionView * n)()
    keep = []
    for i, v in enumerate(views):
        srcs = np.array(v["srcs"], np.int32)
        keep.append(srcs)
        arr[i] = OracleFusionView(v["depth"].shape[1], v["depth"].shape[0], v["cam"], v["depth"].ctypes.data,
                                  v["normal"].ctypes.data, v["weak"].ctypes.data, v["conf"].ctypes.data,
                                  v["bgr"].ctypes.data, v["ref"], len(srcs), srcs.ctypes.data)
    return arr, keep


def oracle_weak_filter(views, ref):
    lib = oracle()
    lib.oracle_weak_vis_filter.argtypes = [C.c_int, C.POINTER(OracleFusionView), C.c_int, C.c_void_p]
    arr, _keep = _oracle_views(views)
    out = np.zeros(views[ref]["depth"].shape, np.uint8)
    lib.oracle_weak_vis_filter(len(views), arr, ref, out.ctypes.data)
    return out


def oracle_candidates(views, ref, src_idx):
    """Per-(pixel, source) sp / dist / rel / angle / q of the reference's loops (no masks)."""
    lib = oracle()
    lib.oracle_fusion_candidates.argtypes = [C.POINTER(OracleFusionView), C.c_int, C.c_int, C.c_void_p] + \
        [C.c_void_p] * 5
    arr, _keep = _oracle_views(views)
    H, W = views[ref]["depth"].shape
    s = np.asarray(src_idx, np.int32)
    shp = (H, W, len(s))
    sp = np.zeros(shp, np.int32)
    f = [np.zeros(shp, np.float32) for _ in range(4)]
    lib.oracle_fusion_candidates(arr, ref, len(s), s.ctypes.data, sp.ctypes.data, *[x.ctypes.data for x in f])
    return sp, f[0], f[1], f[2], f[3]


def run_oracle(views, dataset, weak_filter):
    lib = oracle()
    n = len(views)
    arr = (OracleFusionView * n)()
    keep = []
    for i, v in enumerate(views):
        srcs = np.array(v["srcs"], np.int32)
        keep.append(srcs)
        arr[i] = OracleFusionView(v["depth"].shape[1], v["depth"].shape[0], v["cam"], v["depth"].ctypes.data,
                                  v["normal"].ctypes.data, v["weak"].ctypes.data, v["conf"].ctypes.data,
                                  v["bgr"].ctypes.data, v["ref"], len(srcs), srcs.ctypes.data)
    skips = [np.zeros(v["depth"].shape, np.uint8) for v in views]
    skip_ptrs = (C.c_void_p * n)(*[s.ctypes.data for s in skips])
    cap = sum(v["depth"].size for v in views)
    xyz = np.zeros((cap, 3), np.float32)
    col = np.zeros((cap, 3), np.float32)
    counts = np.zeros(n, np.int64)
    m = lib.oracle_fusion(VARIANTS.get(dataset, 0), n, arr, int(weak_filter), skip_ptrs, xyz.ctypes.data,
                          col.ctypes.data, cap, counts.ctypes.data)
    return xyz[:m].copy(), col[:m].copy(), skips, counts


def ply_bytes(xyz, col, export_color=True):
    """ExportPointCloud (APD.cpp:316-356) in numpy: the expected file content."""
    head = ("ply\nformat binary_little_endian 1.0\n"
            f"element vertex {len(xyz)}\nproperty float x\nproperty float y\nproperty float z\n")
    if export_color:
        head += "property uchar blue\nproperty uchar green\nproperty uchar red\n"
    head += "end_header\n"
    if export_color:
        rec = np.zeros(len(xyz), dtype=[("p", "<f4", 3), ("c", "u1", 3)])
        rec["p"] = xyz
        rec["c"] = col.astype(np.uint8)  # static_cast<uchar>(float): truncation
    else:
        rec = np.ascontiguousarray(xyz, "<f4")
    return head.encode() + rec.tobytes()


def read_ply(path):
    data = open(path, "rb").read()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    head = data[:end].decode()
    n = int([ln for ln in head.split("\n") if ln.startswith("element vertex")][0].split()[-1])
    color = "uchar blue" in head
    dt = np.dtype([("p", "<f4", 3), ("c", "u1", 3)]) if color else np.dtype([("p", "<f4", 3)])
    rec = np.frombuffer(data[end:], dt, count=n)
    return head, rec
