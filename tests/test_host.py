"""CPU tests of the host side of the drop-in (apde-mvs_amd/host): image decoding vs Pillow, OpenCV-rule
resizing, cam.txt parsing, and the `apd` binary's command-line contract (main.cpp:9-40)."""
import ctypes as C
import io
import os
import subprocess

import numpy as np
import pytest
from PIL import Image

import apd_abi as A
import host_schedule as HS

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(REPO, "apde-mvs_amd", "host")
APD_BIN = os.path.join(HOST, "build", "apd")
HOST_LIB = os.path.join(HOST, "build", "libapdhost.so")


@pytest.fixture(scope="module")
def hostlib():
    if not os.path.exists(os.path.join(REPO, "apde-mvs_amd", "lib", "libapd_hip.so")):
        subprocess.run(["make", "-C", os.path.join(REPO, "apde-mvs_amd")], check=True, capture_output=True)
    subprocess.run(["make", "-C", HOST], check=True, capture_output=True)
    A.torch_runtime_first()  # libapdhost.so links libapd_hip.so
    lib = C.CDLL(HOST_LIB)
    lib.apdhost_read_gray8.restype = C.c_long
    lib.apdhost_read_gray8.argtypes = [C.c_char_p, C.c_void_p, C.c_long, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    lib.apdhost_resize_linear_f32.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int]
    lib.apdhost_resize_nearest.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int]
    lib.apdhost_read_camera.restype = C.c_int
    lib.apdhost_read_camera.argtypes = [C.c_char_p, C.POINTER(A.ApdCamera)]
    lib.apdhost_read_binmat.restype = C.c_long
    lib.apdhost_read_binmat.argtypes = [C.c_char_p, C.c_void_p, C.c_long] + [C.POINTER(C.c_int)] * 3
    return lib


def decode(lib, path):
    w, h = C.c_int(), C.c_int()
    n = lib.apdhost_read_gray8(path.encode(), None, 0, C.byref(w), C.byref(h))
    assert n > 0, f"decode failed: {path}"
    out = np.zeros(n, np.uint8)
    lib.apdhost_read_gray8(path.encode(), out.ctypes.data, n, C.byref(w), C.byref(h))
    return out.reshape(h.value, w.value)


def textured(h, w, seed=0, ch=1):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    base = 128 + 60 * np.sin(xx / 7.0) * np.cos(yy / 11.0) + rng.normal(0, 20, (h, w))
    if ch == 1:
        return np.clip(base, 0, 255).astype(np.uint8)
    return np.clip(np.stack([base + 30 * k + rng.normal(0, 10, (h, w)) for k in range(ch)], -1), 0, 255).astype(np.uint8)


def libpng_gray(rgb):
    r, g, b = (rgb[..., k].astype(np.int64) for k in range(3))
    out = (9798 * r + 19235 * g + 3735 * b) >> 15
    same = (r == g) & (r == b)
    return np.where(same, r, out).astype(np.uint8)


@pytest.mark.parametrize("mode", ["L", "LA", "RGB", "RGBA", "P"])
def test_png_decode(hostlib, tmp_path, mode):
    h, w = 37, 53
    if mode in ("L", "LA"):
        img = Image.fromarray(textured(h, w), "L").convert(mode)
    else:
        img = Image.fromarray(textured(h, w, ch=3), "RGB").convert(mode)
    p = str(tmp_path / "x.png")
    img.save(p, optimize=(mode == "L"))
    got = decode(hostlib, p)
    if mode in ("L", "LA"):
        exp = np.asarray(img.convert("L"))
    elif mode == "P":
        exp = libpng_gray(np.asarray(img.convert("RGB")))
    else:
        exp = libpng_gray(np.asarray(img)[..., :3])
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("kind,quality,sub", [("L", 75, 0), ("L", 95, 0), ("RGB", 90, 0), ("RGB", 75, 2),
                                                ("RGB", 50, 1)])
def test_jpeg_luma_matches_libjpeg(hostlib, tmp_path, kind, quality, sub):
    """Baseline JPEG luma plane == libjpeg's JCS_GRAYSCALE output (Pillow draft mode 'L')."""
    img = Image.fromarray(textured(45, 67, ch=1 if kind == "L" else 3), kind)
    p = str(tmp_path / "x.jpg")
    img.save(p, quality=quality, subsampling=sub)
    ref = Image.open(p)
    ref.draft("L", ref.size)
    exp = np.asarray(ref.convert("L") if ref.mode != "L" else ref)
    got = decode(hostlib, p)
    assert got.shape == exp.shape
    assert np.array_equal(got, exp), f"max diff {np.abs(got.astype(int) - exp.astype(int)).max()}"


def test_jpeg_restart_markers(hostlib, tmp_path):
    img = Image.fromarray(textured(64, 96, ch=3), "RGB")
    p = str(tmp_path / "r.jpg")
    try:
        img.save(p, quality=85, restart_marker_blocks=3)
    except TypeError:
        pytest.skip("this Pillow cannot write restart markers")
    data = open(p, "rb").read()
    if b"\xff\xdd" not in data:
        pytest.skip("this Pillow ignored restart_marker_blocks")
    ref = Image.open(p)
    ref.draft("L", ref.size)
    assert np.array_equal(decode(hostlib, p), np.asarray(ref.convert("L")))


def test_pgm_decode(hostlib, tmp_path):
    img = textured(20, 31)
    p = str(tmp_path / "x.pgm")
    with open(p, "wb") as fh:
        fh.write(b"P5\n# comment\n31 20\n255\n" + img.tobytes())
    assert np.array_equal(decode(hostlib, p), img)


def test_unsupported_image_fails(hostlib, tmp_path):
    p = str(tmp_path / "x.jpg")
    Image.fromarray(textured(16, 16, ch=3), "RGB").save(p, progressive=True)
    w, h = C.c_int(), C.c_int()
    assert hostlib.apdhost_read_gray8(p.encode(), None, 0, C.byref(w), C.byref(h)) < 0


def resize_c(lib, img, w, h):
    src = np.ascontiguousarray(img, np.float32)
    dst = np.zeros((h, w), np.float32)
    lib.apdhost_resize_linear_f32(src.ctypes.data, src.shape[1], src.shape[0], dst.ctypes.data, w, h)
    return dst


@pytest.mark.parametrize("sw,sh,dw,dh", [(64, 48, 32, 24), (64, 48, 16, 12), (64, 48, 8, 6), (100, 60, 37, 23),
                                         (30, 20, 45, 31), (64, 48, 64, 48)])
def test_resize_linear(hostlib, sw, sh, dw, dh):
    img = textured(sh, sw).astype(np.float32)
    got = resize_c(hostlib, img, dw, dh)
    assert np.array_equal(got, HS.resize_linear(img, dw, dh))


def test_resize_known_answers(hostlib):
    img = textured(48, 64).astype(np.float32)
    half = resize_c(hostlib, img, 32, 24)  # exact 2x: INTER_AREA mean of each 2x2 block
    exp = img.reshape(24, 2, 32, 2).mean(axis=(1, 3))
    assert np.array_equal(half, exp.astype(np.float32))
    q = resize_c(hostlib, img, 16, 12)  # 4x INTER_LINEAR: mean of the centre 2x2 of each 4x4 block
    exp4 = img.reshape(12, 4, 16, 4)[:, 1:3, :, 1:3].mean(axis=(1, 3))
    assert np.array_equal(q, exp4.astype(np.float32))


def test_resize_nearest(hostlib):
    m = np.arange(48 * 64, dtype=np.float32).reshape(48, 64)
    for (w, h) in [(32, 24), (100, 70), (17, 9)]:
        dst = np.zeros((h, w), np.float32)
        hostlib.apdhost_resize_nearest(m.ctypes.data, 64, 48, dst.ctypes.data, w, h, 4)
        assert np.array_equal(dst, HS.resize_nearest(m, w, h))


def test_read_camera(hostlib, tmp_path):
    p = str(tmp_path / "00000000_cam.txt")
    with open(p, "w") as fh:
        fh.write("extrinsic\n0.1 0.2 0.3 1.5\n0.4 0.5 0.6 -2.25\n0.7 0.8 0.9 3.125\n0 0 0 1\n\n"
                 "intrinsic\n1000.5 0 320.25\n0 999.75 240.5\n0 0 1\n\n0.5 0.01\n")
    cam = A.ApdCamera()
    assert hostlib.apdhost_read_camera(p.encode(), C.byref(cam)) == 0
    exp = HS.read_cam(p)
    assert np.array_equal(np.array(cam.K[:], np.float32), exp["K"])
    assert np.array_equal(np.array(cam.R[:], np.float32), exp["R"])
    assert np.array_equal(np.array(cam.c[:], np.float32), exp["c"])
    assert cam.depth_num == 192.0  # fallback (APD.cpp:128-131)
    assert np.float32(cam.depth_max) == exp["depth_max"]


def run_apd(*args, timeout=60):
    return subprocess.run([APD_BIN, *args], capture_output=True, text=True, timeout=timeout)


def test_cli_help_and_errors(hostlib):
    r = run_apd("-h")
    assert r.returncode == 0 and "--dense_folder" in r.stdout and "--memory_cache" in r.stdout
    r = run_apd()
    assert r.returncode == 255 and "Error:" in r.stdout and "dense_folder" in r.stdout
    r = run_apd("--dense_folder", "/nonexistent", "--use_sa", "maybe")
    assert r.returncode == 255 and "invalid" in r.stdout
    r = run_apd("--dense_folder", "/nonexistent", "--bogus", "1")
    assert r.returncode == 255


def test_cli_bad_scan_folder(hostlib, tmp_path):
    r = run_apd("--dense_folder", str(tmp_path), "--no_fuse", "true")
    assert r.returncode != 0


def test_binmat_read_and_truncation(hostlib, tmp_path):
    """ReadBinMat (APD.cpp:18-56): a complete file reads back; a truncated one is rejected as a whole
    (no partly filled Mat whose tail would hold another problem's pooled bytes)."""
    import synth
    m = np.arange(37 * 23, dtype=np.float32).reshape(23, 37)
    path = str(tmp_path / "d.bin")
    synth.write_bin_mat(path, m)
    r, c, t = C.c_int(), C.c_int(), C.c_int()
    out = np.zeros_like(m)
    n = hostlib.apdhost_read_binmat(path.encode(), out.ctypes.data, out.nbytes, C.byref(r), C.byref(c), C.byref(t))
    assert n == m.nbytes and (r.value, c.value, t.value) == (23, 37, 5) and np.array_equal(out, m)
    data = open(path, "rb").read()
    for cut in (8, 16, 17, len(data) // 2, len(data) - 1):
        open(path, "wb").write(data[:cut])
        assert hostlib.apdhost_read_binmat(path.encode(), None, 0, C.byref(r), C.byref(c), C.byref(t)) == -1, cut
