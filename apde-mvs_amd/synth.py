"""Seeded synthetic piecewise-planar scenes in the MVSNet scan layout.

Stands in for ETH3D / Tanks&Temples data, which are not available offline:
a back wall, a floor and slanted boxes, each textured with band-limited noise, plus large
constant-intensity patches that force WEAK (textureless) pixels. N+1 pinhole cameras with
f = 0.8*W, principal point at the centre, sources on an arc with baselines of 5-15 % of the median
depth looking at the scene centre. The scan layout (cams/%08d_cam.txt, images/, pair.txt) is the one
tools/colmap2mvsnet.py:494-514 writes and APD.cpp:85-135 / main.cpp:44-102 read.
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import numpy as np


@dataclass
class Camera:
    K: np.ndarray  # 3x3
    R: np.ndarray  # 3x3 world->camera
    t: np.ndarray  # 3
    depth_min: float = 0.0
    depth_max: float = 1.0
    interval: float = 0.0
    depth_num: float = 192.0

    @property
    def center(self) -> np.ndarray:
        return -self.R.T @ self.t


@dataclass
class Scene:
    width: int
    height: int
    images: list  # float32 HxW, values are integers 0..255
    cameras: list  # Camera
    gt_depth: list  # float32 HxW per view (0 = no surface)
    labels: list  # uint8 HxW per view: plane id + 1 (SA mask stand-in)
    pairs: list = field(default_factory=list)  # per view: list of (src_id, score)


def _look_at(center, target, up=np.array([0.0, -1.0, 0.0])):
    z = target - center
    z = z / np.linalg.norm(z)
    x = np.cross(z, up)
    x = x / np.linalg.norm(x)
    y = np.cross(z, x)
    R = np.stack([x, y, z], axis=0)
    t = -R @ center
    return R, t


class _Texture:
    """Band-limited noise: a seeded FFT-filtered tileable noise image, sampled bilinearly (wrap) at
    in-plane coordinates, so every view sees the same surface texture."""

    SIZE = 512

    def __init__(self, rng, base_freq=6.0, flat_patches=(), detail=None, scale=1.0):
        n = self.SIZE
        self.tex = self._noise(rng, n, 24.0)  # keep ~24 cycles per tile
        self.k = base_freq * n / 24.0 / (2 * np.pi) * 2.0 / scale  # texels per world unit
        self.flat = list(flat_patches)  # (u0, v0, u1, v1, value)
        self.mean = rng.uniform(90, 160)
        self.scale = rng.uniform(28, 40)
        # optional fine detail (texture-rich scenes): (rng, texels per world unit, amplitude), from a
        # generator of its own so the coarse texture is the same with and without it
        self.detail = None
        if detail is not None:
            drng, dk, damp = detail
            self.detail = (self._noise(drng, self.DETAIL_SIZE, self.DETAIL_SIZE / 8.0), dk, damp)

    DETAIL_SIZE = 1024

    @staticmethod
    def _noise(rng, n, cycles):
        white = rng.normal(size=(n, n))
        fy = np.fft.fftfreq(n)[:, None]
        fx = np.fft.fftfreq(n)[None, :]
        band = np.exp(-((np.hypot(fx, fy) * n / cycles) ** 2))
        tex = np.real(np.fft.ifft2(np.fft.fft2(white) * band))
        return (tex / tex.std()).astype(np.float32)

    @staticmethod
    def _bilinear(T, x, y):
        n = T.shape[0]
        x0 = np.floor(x)
        y0 = np.floor(y)
        ax = x - x0
        ay = y - y0
        x0 = x0.astype(np.int64) % n
        y0 = y0.astype(np.int64) % n
        x1 = (x0 + 1) % n
        y1 = (y0 + 1) % n
        top = T[y0, x0] * (1 - ax) + T[y0, x1] * ax
        bot = T[y1, x0] * (1 - ax) + T[y1, x1] * ax
        return top * (1 - ay) + bot * ay

    def __call__(self, u, v):
        """Returns (value, flat_mask): flat_mask marks the textureless patches."""
        val = self.mean + self.scale * self._bilinear(self.tex, u * self.k, v * self.k)
        if self.detail is not None:
            T, dk, damp = self.detail
            val = val + damp * self.scale * self._bilinear(T, u * dk, v * dk)
        flat = np.zeros(val.shape, bool)
        for (u0, v0, u1, v1, value) in self.flat:
            m = (u >= u0) & (u <= u1) & (v >= v0) & (v <= v1)
            val = np.where(m, value, val)
            flat |= m
        return val, flat


class _Quad:
    """A bounded planar patch: origin + s*eu + t*ev, s,t in [0,1]."""

    def __init__(self, origin, eu, ev, tex):
        self.o = np.asarray(origin, float)
        self.eu = np.asarray(eu, float)
        self.ev = np.asarray(ev, float)
        n = np.cross(self.eu, self.ev)
        self.n = n / np.linalg.norm(n)
        self.tex = tex
        G = np.array([[self.eu @ self.eu, self.eu @ self.ev], [self.eu @ self.ev, self.ev @ self.ev]])
        self.Ginv = np.linalg.inv(G)

    def intersect(self, C, M, xs, ys):
        """Ray cast for pixel rays D(x,y) = M @ (x, y, 1) from centre C. Every dot product of D is
        affine in (x, y), so the whole image is built from broadcast row/column vectors.
        Returns t (inf where missed) and in-plane coordinates (u, v)."""
        def lin(vec):
            w = M.T @ vec
            return w[0] * xs[None, :] + w[1] * ys[:, None] + w[2]

        with np.errstate(divide="ignore", invalid="ignore"):
            t = ((self.o - C) @ self.n) / lin(self.n)
            rel0 = C - self.o
            b0 = rel0 @ self.eu + t * lin(self.eu)
            b1 = rel0 @ self.ev + t * lin(self.ev)
            s = self.Ginv[0, 0] * b0 + self.Ginv[0, 1] * b1
            r = self.Ginv[1, 0] * b0 + self.Ginv[1, 1] * b1
            ok = (t > 1e-6) & (s >= 0) & (s <= 1) & (r >= 0) & (r <= 1) & np.isfinite(t)
        return np.where(ok, t, np.inf), s * np.linalg.norm(self.eu), r * np.linalg.norm(self.ev)


TEXTURES = ("smooth", "rich")


def make_scene(width=160, height=120, num_src=4, seed=20251114, weak_patches=True, depth=6.0,
               workers: int = 0, texture: str = "smooth", detail_period_px: float = 5.0,
               texture_scale: float = 1.0) -> Scene:
    """texture="smooth": band-limited textures fixed in world units, so they get smoother per pixel
    as the resolution grows (90-94 % of the pixels end WEAK at 3024x2016 and 6048x4032).
    texture="rich": the same scene plus a fine detail octave of `detail_period_px` pixels at the
    reference view, and two more textureless patches: a resolution-independent, texture-rich
    variant whose WEAK fraction is set by the textureless area.
    texture_scale: the smooth textures' world wavelengths times this factor. A scene rendered at
    1/s of a resolution with texture_scale s has that resolution's texture per pixel (its WEAK
    fraction): bench.py's CPU baseline samples the C3 workload that way. The random draws do not
    change, so texture_scale = 1 is the scene of every other caller."""
    if texture not in TEXTURES:
        raise ValueError(f"texture must be one of {TEXTURES}")
    rng = np.random.default_rng(seed)
    rich = texture == "rich"
    drng = np.random.default_rng(seed + 1) if rich else None
    f = 0.8 * width
    K = np.array([[f, 0.0, width / 2.0], [0.0, f, height / 2.0], [0.0, 0.0, 1.0]])

    def detail():
        if not rich:
            return None
        period_world = detail_period_px * depth / f  # world size of the detail period at the wall
        return (drng, (_Texture.DETAIL_SIZE / (_Texture.DETAIL_SIZE / 8.0)) / period_world, 0.8)

    # scene geometry in world coords (ref camera at origin looking along +z)
    half_w = depth * (width / 2.0) / f * 1.6
    half_h = depth * (height / 2.0) / f * 1.6
    quads = []
    flat = [(0.68 * half_w, 0.25 * half_h, 1.2 * half_w, 1.1 * half_h, 128.0)] if weak_patches else []
    floor_flat = []
    if rich and weak_patches:
        flat += [(1.45 * half_w, 0.1 * half_h, 2.0 * half_w, 1.5 * half_h, 112.0)]
        floor_flat = [(0.2 * half_w, 0.0, 1.1 * half_w, 0.35 * depth, 96.0)]
    quads.append(_Quad([-half_w, -half_h, depth], [2 * half_w, 0, 0.35 * depth], [0, 2 * half_h, 0],
                       _Texture(rng, base_freq=4.0, flat_patches=flat, detail=detail(), scale=texture_scale)))  # slanted back wall
    quads.append(_Quad([-half_w, 0.55 * half_h, 0.45 * depth], [2 * half_w, 0, 0],
                       [0, 0.45 * half_h, 0.9 * depth],
                       _Texture(rng, base_freq=5.0, flat_patches=floor_flat, detail=detail(), scale=texture_scale)))  # floor
    for b in range(3):
        cx = rng.uniform(-0.6, 0.6) * half_w
        cy = rng.uniform(-0.5, 0.3) * half_h
        cz = rng.uniform(0.6, 0.85) * depth
        sz = rng.uniform(0.15, 0.3) * half_w
        ang = rng.uniform(-0.6, 0.6)
        eu = np.array([np.cos(ang), 0, np.sin(ang)]) * sz
        ev = np.array([0, 1.0, rng.uniform(-0.3, 0.3)]) * sz
        bflat = [(0.1 * sz, 0.1 * sz, 0.7 * sz, 0.7 * sz, rng.uniform(60, 200))] if (weak_patches and b == 0) else []
        quads.append(_Quad([cx, cy, cz], eu, ev, _Texture(rng, base_freq=7.0, flat_patches=bflat, detail=detail(), scale=texture_scale)))

    # cameras: ref at origin, sources on an arc around the scene centre
    target = np.array([0.0, 0.0, 0.8 * depth])
    cams = [Camera(K.copy(), np.eye(3), np.zeros(3))]
    for i in range(num_src):
        ang = (i + 1) / (num_src + 1) * 2 * np.pi
        base = rng.uniform(0.05, 0.15) * depth
        C = np.array([np.cos(ang) * base, np.sin(ang) * base * 0.6, rng.uniform(-0.03, 0.03) * depth])
        R, t = _look_at(C, target + rng.normal(size=3) * 0.02 * depth)
        cams.append(Camera(K.copy(), R, t))

    xs = np.arange(width, dtype=np.float64)
    ys = np.arange(height, dtype=np.float64)
    Kinv = np.linalg.inv(K)

    def render(cam, noise):
        M = cam.R.T @ Kinv  # world-frame ray of pixel (x, y) with camera-frame z = 1
        C = cam.center
        best_t = np.full((height, width), np.inf)
        best_q = np.full((height, width), -1, np.int64)
        hits = []
        for qi, q in enumerate(quads):
            t, s, r = q.intersect(C, M, xs, ys)
            closer = t < best_t
            best_t = np.where(closer, t, best_t)
            best_q = np.where(closer, qi, best_q)
            hits.append((s, r))
        val = np.zeros((height, width))
        flat = np.zeros((height, width), bool)
        for qi, q in enumerate(quads):
            m = best_q == qi
            if m.any():
                tv, tf = q.tex(hits[qi][0][m], hits[qi][1][m])
                val[m] = tv
                flat[m] = tf
        del hits
        lab = (best_q + 1).astype(np.uint8)
        hit = np.isfinite(best_t)
        # textureless patches: constant albedo + per-view sensor noise (uncorrelated across views, so
        # NCC cannot lock on and DepthToWeak classifies them WEAK, APD.cu:2220-2249)
        val = np.where(flat, val + noise, val)
        img = np.where(hit, val, 30.0)
        img = np.clip(np.round(img), 0, 255).astype(np.float32)
        return img, np.where(hit, best_t, 0.0).astype(np.float32), lab  # ray z = 1 in camera frame

    # The views render in parallel (numpy releases the GIL in its array loops); the only random draws
    # after the cameras are each view's sensor noise, drawn here in view order, so the scene does not
    # depend on the number of workers.
    workers = max(1, min(len(cams), workers if workers else min(8, os.cpu_count() or 1)))
    with ThreadPoolExecutor(workers) as pool:
        futs = [pool.submit(render, cam, rng.normal(0.0, 2.0, size=(height, width))) for cam in cams]
        rendered = [f.result() for f in futs]
    images = [r[0] for r in rendered]
    depths = [r[1] for r in rendered]
    labels = [r[2] for r in rendered]
    del rendered
    valid = np.concatenate([d[d > 0] for d in depths])
    dmin = float(np.percentile(valid, 1) * 0.75)
    dmax = float(np.percentile(valid, 99) * 1.25)
    for cam in cams:
        cam.depth_min, cam.depth_max = dmin, dmax
        cam.depth_num = 192.0
        cam.interval = (dmax - dmin) / 192.0
    nv = len(cams)
    pairs = []
    for i in range(nv):
        others = [j for j in range(nv) if j != i]
        dists = [np.linalg.norm(cams[i].center - cams[j].center) for j in others]
        order = [others[k] for k in np.argsort(dists)]
        pairs.append([(j, float(nv - r)) for r, j in enumerate(order)])
    return Scene(width, height, images, cams, depths, labels, pairs)


def camera_struct_values(cam: Camera, width: int, height: int):
    """Field values of apd_camera / Camera (main.h:50-61), c computed as APD.cpp:114-119."""
    R = cam.R.astype(np.float32)
    t = cam.t.astype(np.float32)
    c = np.array([-(float(np.float64(R[0, j]) * t[0] + np.float64(R[1, j]) * t[1] + np.float64(R[2, j]) * t[2]))
                  for j in range(3)], np.float32)
    return dict(K=cam.K.astype(np.float32).ravel(), R=R.ravel(), t=t, c=c, height=height, width=width,
                depth_min=np.float32(cam.depth_min), depth_max=np.float32(cam.depth_max),
                interval=np.float32(cam.interval), depth_num=np.float32(cam.depth_num))


def write_scan(scene: Scene, folder: str, ext: str = ".pgm", write_masks: bool = False) -> None:
    """Write the MVSNet scan layout read by the reference (APD.cpp:85-135, main.cpp:44-102)."""
    os.makedirs(os.path.join(folder, "images"), exist_ok=True)
    os.makedirs(os.path.join(folder, "cams"), exist_ok=True)
    for i, (img, cam) in enumerate(zip(scene.images, scene.cameras)):
        name = f"{i:08d}"
        write_pgm(os.path.join(folder, "images", name + ext), img.astype(np.uint8))
        with open(os.path.join(folder, "cams", name + "_cam.txt"), "w") as fh:
            fh.write("extrinsic\n")
            for r in range(3):
                fh.write(" ".join(repr(float(v)) for v in cam.R[r]) + " " + repr(float(cam.t[r])) + "\n")
            fh.write("0.0 0.0 0.0 1.0\n\nintrinsic\n")
            for r in range(3):
                fh.write(" ".join(repr(float(v)) for v in cam.K[r]) + "\n")
            fh.write(f"\n{cam.depth_min!r} {cam.interval!r} {cam.depth_num!r} {cam.depth_max!r}\n")
    with open(os.path.join(folder, "pair.txt"), "w") as fh:
        fh.write(f"{len(scene.images)}\n")
        for i, pl in enumerate(scene.pairs):
            fh.write(f"{i}\n{len(pl)} " + " ".join(f"{j} {s}" for j, s in pl) + "\n")
    if write_masks:
        os.makedirs(os.path.join(folder, "sa_masks"), exist_ok=True)
        for i, lab in enumerate(scene.labels):
            write_bin_mat(os.path.join(folder, "sa_masks", f"{i:08d}.bin"), lab)


def write_pgm(path: str, img_u8: np.ndarray) -> None:
    h, w = img_u8.shape
    with open(path, "wb") as fh:
        fh.write(f"P5\n{w} {h}\n255\n".encode())
        fh.write(np.ascontiguousarray(img_u8, np.uint8).tobytes())


_CV_TYPES = {(np.dtype(np.uint8), 1): 0, (np.dtype(np.int32), 1): 4, (np.dtype(np.float32), 1): 5,
             (np.dtype(np.float32), 3): 21}


def write_bin_mat(path: str, mat: np.ndarray) -> None:
    """WriteBinMat, APD.cpp:58-83: int32 version=1, rows, cols, cv type, raw row-major data."""
    ch = 1 if mat.ndim == 2 else mat.shape[2]
    cvt = _CV_TYPES[(mat.dtype, ch)]
    with open(path, "wb") as fh:
        np.array([1, mat.shape[0], mat.shape[1], cvt], np.int32).tofile(fh)
        fh.write(np.ascontiguousarray(mat).tobytes())


def read_bin_mat(path: str) -> np.ndarray:
    """ReadBinMat, APD.cpp:18-56."""
    with open(path, "rb") as fh:
        hdr = np.frombuffer(fh.read(16), np.int32)
        version, rows, cols, cvt = (int(v) for v in hdr)
        if version != 1:
            raise ValueError(f"bin-mat version {version} != 1: {path}")
        dt, ch = {0: (np.uint8, 1), 4: (np.int32, 1), 5: (np.float32, 1), 21: (np.float32, 3)}[cvt]
        data = np.frombuffer(fh.read(), dt)
    return data.reshape((rows, cols) if ch == 1 else (rows, cols, ch)).copy()
