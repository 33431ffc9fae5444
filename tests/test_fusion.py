"""Fusion (RunFusion / RunFusion_TAT_I / RunFusion_TAT_A + WeakVisFilter, APD.cpp:962-1608).

CPU: the oracle (oracle/fusion_oracle.c) against analytic known answers, the exact angle cuts the
kernels compare against, and the colour decode (cv::imread IMREAD_COLOR) against libjpeg/libpng
through Pillow. GPU: the `apd --only_fuse` binary (HIP kernels + host ordered commit) must write
byte-identical APD.ply and identical skip.png maps to the oracle on the same scan.

Parity of the oracle with the reference binary is unpinned: the reference needs CUDA + OpenCV to
build and ships no fusion fixtures.
"""
import ctypes as C
import math
import os
import shutil
import subprocess

import numpy as np
import pytest
from PIL import Image

import apd_abi as A
import fusion_lib as FL
import synth

LIBM = C.CDLL("libm.so.6")
LIBM.acosf.restype = C.c_float
LIBM.acosf.argtypes = [C.c_float]


def f32(x):
    return float(np.float32(x))


def next_up(x):
    return float(np.nextafter(np.float32(x), np.float32(2)))


def next_down(x):
    return float(np.nextafter(np.float32(x), np.float32(-2)))


@pytest.fixture(scope="module")
def hl():
    return FL.hostlib()


# ------------------------------------------------------------------------------------------------
# exact angle cuts
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("T", [0.174533, 0.06981317007977318 + 2 * 0.05235987755982988,
                               0.06981317007977318 + 5 * 0.05235987755982988, 1.0])
def test_angle_cut(hl, T):
    T = f32(T)
    q = hl.apdhost_angle_cut_lt(T)
    assert LIBM.acosf(q) >= T
    assert LIBM.acosf(next_up(q)) < T


def test_view_cut(hl):
    q = hl.apdhost_view_cut_deg(80.0)

    def deg(v):
        return f32(f32(LIBM.acosf(v) * f32(180.0)) / math.pi)
    assert deg(q) <= 80.0
    assert deg(next_down(q)) > 80.0


# ------------------------------------------------------------------------------------------------
# colour decode (RunFusion reads IMREAD_COLOR, APD.cpp:1077)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("sub", [0, 1, 2])
@pytest.mark.parametrize("size", [(64, 48), (61, 37)])
def test_jpeg_colour_matches_libjpeg(hl, tmp_path, sub, size):
    rng = np.random.default_rng(sub + size[0])
    w, h = size
    yy, xx = np.mgrid[0:h, 0:w]
    rgb = np.stack([(xx * 4) % 256, (yy * 5) % 256, rng.integers(0, 256, (h, w))], -1).astype(np.uint8)
    p = str(tmp_path / "c.jpg")
    Image.fromarray(rgb, "RGB").save(p, quality=90, subsampling=sub)
    got = FL.read_bgr(hl, p)
    ref = np.asarray(Image.open(p).convert("RGB"))[..., ::-1]
    assert np.array_equal(got, ref)


def test_jpeg_gray_as_colour(hl, tmp_path):
    g = (np.arange(40 * 30).reshape(30, 40) % 251).astype(np.uint8)
    p = str(tmp_path / "g.jpg")
    Image.fromarray(g, "L").save(p, quality=85)
    got = FL.read_bgr(hl, p)
    ref = np.asarray(Image.open(p).convert("L"))
    assert np.array_equal(got, np.repeat(ref[..., None], 3, -1))


@pytest.mark.parametrize("mode", ["RGB", "RGBA", "L", "P"])
def test_png_colour(hl, tmp_path, mode):
    rng = np.random.default_rng(3)
    rgb = rng.integers(0, 256, (23, 31, 3)).astype(np.uint8)
    img = Image.fromarray(rgb, "RGB")
    if mode != "RGB":
        img = img.convert(mode)
    p = str(tmp_path / "c.png")
    img.save(p)
    got = FL.read_bgr(hl, p)
    ref = np.asarray(Image.open(p).convert("RGB"))[..., ::-1]
    assert np.array_equal(got, ref)


def test_resize_u8c3_area_and_identity(hl):
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (20, 30, 3)).astype(np.uint8)
    assert np.array_equal(FL.resize_bgr(hl, img, 30, 20), img)
    half = FL.resize_bgr(hl, img, 15, 10)  # exact 2x -> INTER_AREA: (a+b+c+d+2) >> 2
    s = img.astype(np.int32)
    exp = (s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2] + 2) >> 2
    assert np.array_equal(half, exp.astype(np.uint8))
    flat = np.full((17, 23, 3), 77, np.uint8)
    assert np.all(FL.resize_bgr(hl, flat, 31, 11) == 77)


def test_png_writer_roundtrip(hl, tmp_path):
    m = (np.arange(35 * 19) % 2 * 255).astype(np.uint8).reshape(19, 35)
    p = str(tmp_path / "skip.png")
    assert hl.apdhost_write_png_gray8(p.encode(), m.ctypes.data, 35, 19) == 0
    assert np.array_equal(np.asarray(Image.open(p)), m)


# ------------------------------------------------------------------------------------------------
# oracle known answers: identical cameras, so every source projection lands on the same pixel,
# the reprojection error is 0 and the normals agree; only the relative depth decides.
# ------------------------------------------------------------------------------------------------
def _same_camera_views(rel_errs, weak_val, srcs_of_view0):
    H, W = 8, len(rel_errs)
    cam = A.ApdCamera()
    for k, v in enumerate([100.0, 0, W / 2, 0, 100.0, H / 2, 0, 0, 1.0]):
        cam.K[k] = v
    for k in (0, 4, 8):
        cam.R[k] = 1.0
    cam.width, cam.height = W, H
    d0 = np.full((H, W), 5.0, np.float32)
    nrm = np.zeros((H, W, 3), np.float32)
    nrm[..., 2] = 1.0
    views = []
    for i in range(1 + len(srcs_of_view0)):
        d = d0 if i == 0 else (d0 * (1.0 + np.asarray(rel_errs, np.float32))[None, :]).astype(np.float32)
        views.append(dict(ref=i, srcs=srcs_of_view0 if i == 0 else [], depth=np.ascontiguousarray(d),
                          normal=nrm, weak=np.full((H, W), weak_val, np.uint8), conf=np.zeros((H, W), np.uint8),
                          bgr=np.full((H, W, 3), 10 * (i + 1), np.uint8), cam=cam))
    return views


def test_oracle_runfusion_known_answer():
    # dynamic = exp(-200 * rel) per consistent source; accept iff > 0.3 (STRONG) / 0.45 (WEAK)
    errs = [0.001, 0.005, 0.008, 0.02]
    xyz, col, _, _ = FL.run_oracle(_same_camera_views(errs, 1, [1]), "ETH3D", False)
    assert len(xyz) == 8 * 2  # columns 0, 1 of each row
    assert np.allclose(col, (10 + 20) / 2)  # ref colour + one source, / (num_consistent + 1)
    xyz, _, _, _ = FL.run_oracle(_same_camera_views(errs, 0, [1]), "ETH3D", False)
    assert len(xyz) == 8 * 1  # WEAK: 0.45 rejects exp(-1)
    xyz, _, _, _ = FL.run_oracle(_same_camera_views(errs, 1, [1, 2]), "ETH3D", False)
    assert len(xyz) == 8 * 2


def test_oracle_tat_known_answer():
    # TAT_A: k = 2 needs both sources with rel < 2/3000; TAT_I also needs angle < 10 deg (angle 0 here)
    errs = [0.0002, 0.0006, 0.001, 0.002]
    for ds in ("TaT_a", "TaT_i"):
        xyz, col, _, counts = FL.run_oracle(_same_camera_views(errs, 1, [1, 2]), ds, False)
        thr = 2 * np.float32(1 / 3000 if ds == "TaT_a" else 1 / 3500)
        exp_cols = sum(1 for e in errs if e < thr)  # rel = e for the reference view
        assert len(xyz) == 8 * exp_cols
        if ds == "TaT_i":
            assert np.allclose(col, (10 + 20 + 30) / 3)
        else:
            assert np.allclose(col, 10)


def test_oracle_weak_filter_only_flags_weak(tmp_path, hl):
    folder = str(tmp_path / "scan")
    FL.make_fusion_scan(folder, 48, 36, 3, seed=5)
    views = FL.load_views(folder, hl)
    _, _, skips, _ = FL.run_oracle(views, "ETH3D", True)
    for v, s in zip(views, skips):
        assert not np.any(s[v["weak"] != 0])
    assert sum(int(s.sum()) for s in skips) > 0


# ------------------------------------------------------------------------------------------------
# GPU: apd --only_fuse == oracle, byte for byte
# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def fusion_scan(tmp_path_factory):
    folder = str(tmp_path_factory.mktemp("fscan"))
    FL.make_fusion_scan(folder, 96, 72, 4, seed=11)
    return folder


def _run_cli(folder, dataset, weak_filter, export_color=True):
    r = subprocess.run([FL.APD_BIN, "--dense_folder", folder, "--dataset", dataset, "--only_fuse", "true",
                        "--weak_filter", str(weak_filter).lower(), "--export_color", str(export_color).lower()],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.gpu
def test_fusion_kernels_match_oracle(fusion_scan, hl):
    """Each device entry point of include/apd_fusion.h against the oracle's literal loops."""
    views = FL.load_views(fusion_scan, hl)
    eng = A.FusionEngine(0)
    eng.set_views(views)
    q_view = hl.apdhost_view_cut_deg(80.0)
    q_angle = hl.apdhost_angle_cut_lt(f32(0.174533))
    ab, ag = f32(0.06981317007977318), f32(0.05235987755982988)
    q_k = [1.0, 1.0] + [hl.apdhost_angle_cut_lt(f32(np.float32(k) * np.float32(ag) + np.float32(ab)))
                        for k in range(2, 33)]
    for i in range(len(views)):
        got = eng.weak_filter(i, q_view)
        exp = FL.oracle_weak_filter(views, i)
        assert np.array_equal(got, exp), f"weak filter view {i}: {int((got != exp).sum())} px differ"
        src = list(range(len(views)))
        src.remove(i)
        sp, dist, rel, ang, q = FL.oracle_candidates(views, i, src)
        live = (views[i]["depth"] > 0)[..., None] & np.ones(len(src), bool)
        valid = sp >= 0
        cons = valid & (dist < 2.0) & (rel < np.float32(0.01)) & (ang < np.float32(0.174533))
        pix, er, qq = eng.consistency(i, src, q_angle)
        exp_pix = np.where(cons, sp, -1)
        bad = (pix != exp_pix) & live
        assert not bad.any(), f"consistency view {i}: {int(bad.sum())} differ, first {np.argwhere(bad)[:3]}"
        chk = valid & live
        assert np.array_equal(er[chk].view(np.uint32), (dist + np.float32(200) * rel)[chk].view(np.uint32))
        assert np.array_equal(qq[chk].view(np.uint32), q[chk].view(np.uint32))
        for tat_i, depth_base in ((True, np.float32(1 / 3500)), (False, np.float32(1 / 3000))):
            tp, lv = eng.tat_levels(i, src, 0.25, float(depth_base), q_k if tat_i else None)
            exp_lv = np.full(sp.shape, 255, np.uint8)
            for k in range(len(src), 1, -1):
                kk = np.float32(k)
                ok = valid & (dist < kk * np.float32(0.25)) & (rel < kk * depth_base)
                if tat_i:
                    ok &= ang < kk * ag + ab
                exp_lv[ok] = k
            assert not ((tp != sp) & live).any(), f"tat src pixels view {i}"
            bad = (lv != exp_lv) & live
            assert not bad.any(), f"tat levels view {i} tat_i={tat_i}: {int(bad.sum())} differ"
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("dataset", ["ETH3D", "TaT_i", "TaT_a"])
@pytest.mark.parametrize("weak_filter", [True, False])
def test_fusion_cli_matches_oracle(fusion_scan, hl, tmp_path, dataset, weak_filter):
    folder = str(tmp_path / "run")
    shutil.copytree(fusion_scan, folder)
    out = _run_cli(folder, dataset, weak_filter)
    assert "Fusion done!" in out
    views = FL.load_views(folder, hl)
    xyz, col, skips, counts = FL.run_oracle(views, dataset, weak_filter)
    assert len(xyz) > 500
    got = open(os.path.join(folder, "APD", "APD.ply"), "rb").read()
    exp = FL.ply_bytes(xyz, col)
    if got != exp:
        head, rec = FL.read_ply(os.path.join(folder, "APD", "APD.ply"))
        pytest.fail(f"APD.ply differs: {len(rec)} points vs {len(xyz)} expected; head {head!r}")
    if weak_filter:
        for v, s in zip(views, skips):
            png = np.asarray(Image.open(os.path.join(folder, "APD", f"{v['ref']:08d}", "skip.png")))
            assert np.array_equal(png, s * 255)
        assert sum(int(s.sum()) for s in skips) > 0
    if dataset == "TaT_a":
        assert [int(ln.split()[-1]) for ln in out.splitlines() if ln.startswith("skip_weak:")] == list(counts)


@pytest.mark.gpu
@pytest.mark.parametrize("scale", [2.0, 1.5])
def test_fusion_cli_rescaled_images(hl, tmp_path, scale):
    """Colour images larger than the depth maps: RescaleImageAndCamera (resize + K scaling)."""
    folder = str(tmp_path / "scan")
    FL.make_fusion_scan(folder, 80, 60, 3, seed=23, image_scale=scale)
    _run_cli(folder, "ETH3D", True, export_color=False)
    views = FL.load_views(folder, hl)
    xyz, col, _, _ = FL.run_oracle(views, "ETH3D", True)
    got = open(os.path.join(folder, "APD", "APD.ply"), "rb").read()
    assert got == FL.ply_bytes(xyz, col, export_color=False)
