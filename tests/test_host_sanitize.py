"""The host parsers (apde-mvs_amd/host: image.cpp's PNG / JPEG / PGM decoders, io.cpp's bin-mat,
cam.txt and pair.txt readers) under AddressSanitizer + UndefinedBehaviorSanitizer, over a corpus of
valid files and corrupt ones derived from them: truncations at many offsets, random byte flips, and
headers claiming huge or zero sizes. Every file must be decoded or rejected -- no out-of-bounds
access, no undefined behaviour (the build aborts on the first report). CPU only."""
import io
import os
import subprocess

import numpy as np
import pytest
from PIL import Image

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(REPO, "apde-mvs_amd", "host")
BIN = os.path.join(HOST, "build-san", "corpus_main")


def _images(rng):
    yy, xx = np.mgrid[0:37, 0:53]
    g = np.clip(128 + 60 * np.sin(xx / 5.0) + rng.normal(0, 20, xx.shape), 0, 255).astype(np.uint8)
    rgb = np.stack([g, np.roll(g, 3, 1), 255 - g], -1)
    out = {}
    for name, img, fmt, kw in [
        ("g.png", Image.fromarray(g), "PNG", {}),
        ("rgb.png", Image.fromarray(rgb), "PNG", {}),
        ("pal.png", Image.fromarray(rgb).convert("P"), "PNG", {}),
        ("g16.png", Image.fromarray((g.astype(np.uint16) * 257)), "PNG", {}),
        ("ga.png", Image.fromarray(g).convert("LA"), "PNG", {}),
        ("g.jpg", Image.fromarray(g), "JPEG", {"quality": 90}),
        ("c420.jpg", Image.fromarray(rgb), "JPEG", {"quality": 75, "subsampling": 2}),
        ("c444.jpg", Image.fromarray(rgb), "JPEG", {"quality": 95, "subsampling": 0}),
        ("rst.jpg", Image.fromarray(rgb), "JPEG", {"quality": 80, "restart_marker_blocks": 2}),
    ]:
        b = io.BytesIO()
        try:
            img.save(b, fmt, **kw)
        except TypeError:
            kw.pop("restart_marker_blocks", None)
            img.save(b, fmt, **kw)
        out[name] = b.getvalue()
    out["g.pgm"] = b"P5\n53 37\n255\n" + g.tobytes()
    out["huge.pgm"] = b"P5\n100000 100000\n255\n" + g.tobytes()
    out["zero.pgm"] = b"P5\n0 0\n255\n"
    binmat = np.array([1, 37, 53, 0], np.int32).tobytes() + g.tobytes()
    out["m.bin"] = binmat
    out["huge.bin"] = np.array([1, 1 << 20, 1 << 20, 5], np.int32).tobytes() + g.tobytes()
    out["neg.bin"] = np.array([1, -5, 7, 5], np.int32).tobytes()
    out["cam.txt"] = (b"extrinsic\n1 0 0 0\n0 1 0 0\n0 0 1 0\n0 0 0 1\n\nintrinsic\n500 0 26\n0 500 18\n0 0 1\n\n"
                      b"1.0 0.01 192 3.0\n")
    return out


def test_host_parsers_under_sanitizers(tmp_path):
    r = subprocess.run(["make", "-C", HOST, "sanitize"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    rng = np.random.default_rng(1)
    files = []
    for name, data in _images(rng).items():
        variants = {"": data}
        for k, cut in enumerate(sorted(set(np.linspace(1, len(data) - 1, 24).astype(int).tolist()))):
            variants[f".cut{k}"] = data[:cut]
        for k in range(24):
            b = bytearray(data)
            for _ in range(int(rng.integers(1, 6))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            variants[f".flip{k}"] = bytes(b)
        for suffix, blob in variants.items():
            p = tmp_path / (name + suffix)
            p.write_bytes(blob)
            files.append(str(p))
    scan = tmp_path / "scan"
    (scan / "images").mkdir(parents=True)
    (scan / "pair.txt").write_bytes(b"3\n0\n2 1 5.0 2 3.0\n1\n2 0 5.0 2 1.0\n2\n999999\n")
    files.append(str(scan))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([BIN, *files], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-3000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    assert "corpus:" in r.stdout
