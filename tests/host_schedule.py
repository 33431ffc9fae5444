"""Python restatement of the reference's host schedule, used as the checker of the `apd` binary.

main.cpp:290-367 (rounds: FIRST_INIT / REFINE_INIT pass + 3 geometric REFINE_ITER passes per round,
scale 2^(rounds-1-i)), APD::InuputInitialization (APD.cpp:501-685: depth range x0.6 / x1.2, image
resize + K scaling, INTER_NEAREST priors, anchors_map) and ProcessProblem's epilogue
(main.cpp:163-178), driving one engine (the HIP library through apd_abi, or the oracle) view by view
in pair.txt order (the reference's sequential ordering) or with pass-start snapshots (jacobi).
Test infrastructure only.
"""
from __future__ import annotations

import math
import os

import numpy as np

import apd_abi as A
import synth

F32 = np.float32


def write_dense_folder(scene, folder, ext=".png", masks=False):
    """MVSNet scan layout with every camera value already float32 (no double rounding on parse)."""
    from PIL import Image
    os.makedirs(os.path.join(folder, "images"), exist_ok=True)
    os.makedirs(os.path.join(folder, "cams"), exist_ok=True)
    r32 = lambda v: repr(float(F32(v)))
    for i, (img, cam) in enumerate(zip(scene.images, scene.cameras)):
        name = f"{i:08d}"
        u8 = np.asarray(img).astype(np.uint8)
        if ext == ".pgm":
            synth.write_pgm(os.path.join(folder, "images", name + ext), u8)
        else:
            Image.fromarray(u8, mode="L").save(os.path.join(folder, "images", name + ext))
        with open(os.path.join(folder, "cams", name + "_cam.txt"), "w") as fh:
            fh.write("extrinsic\n")
            for r in range(3):
                fh.write(" ".join(r32(v) for v in cam.R[r]) + " " + r32(cam.t[r]) + "\n")
            fh.write("0.0 0.0 0.0 1.0\n\nintrinsic\n")
            for r in range(3):
                fh.write(" ".join(r32(v) for v in cam.K[r]) + "\n")
            fh.write(f"\n{r32(cam.depth_min)} {r32(cam.interval)} {r32(cam.depth_num)} {r32(cam.depth_max)}\n")
    with open(os.path.join(folder, "pair.txt"), "w") as fh:
        fh.write(f"{len(scene.images)}\n")
        for i, pl in enumerate(scene.pairs):
            fh.write(f"{i}\n{len(pl)} " + " ".join(f"{j} {s}" for j, s in pl) + "\n")
    if masks:
        os.makedirs(os.path.join(folder, "sa_masks"), exist_ok=True)
        for i, lab in enumerate(scene.labels):
            synth.write_bin_mat(os.path.join(folder, "sa_masks", f"{i:08d}.bin"), lab.astype(np.uint8))


def read_cam(path):
    """ReadCamera (APD.cpp:85-135) with float32 parsing; c = -R^T t in double."""
    tok = open(path).read().split()
    vals = [t for t in tok if t not in ("extrinsic", "intrinsic")]
    f = [F32(float(v)) for v in vals]
    R = np.array([f[0], f[1], f[2], f[4], f[5], f[6], f[8], f[9], f[10]], F32)
    t = np.array([f[3], f[7], f[11]], F32)
    K = np.array(f[16:25], F32)
    c = np.array([-(float(np.float64(R[j]) * np.float64(t[0]) + np.float64(R[3 + j]) * np.float64(t[1])
                          + np.float64(R[6 + j]) * np.float64(t[2]))) for j in range(3)], F32)
    rest = f[25:]
    dmin, interval = rest[0], rest[1]
    if len(rest) >= 4:
        dnum, dmax = rest[2], rest[3]
    else:
        dnum = F32(192)
        dmax = F32(interval * dnum + dmin)
    return dict(K=K, R=R, t=t, c=c, depth_min=dmin, depth_max=dmax, interval=interval, depth_num=dnum)


def resize_linear(img, w, h):
    """cv::resize INTER_LINEAR on CV_32F for the 2^-k pyramid: exact 2x -> INTER_AREA mean, else the
    OpenCV coefficient rule (same arithmetic order as apde-mvs_amd/host/image.cpp)."""
    sh, sw = img.shape
    if sw == w and sh == h:
        return img.copy()
    if sw == 2 * w and sh == 2 * h:
        a = img[0::2, 0::2]; b = img[0::2, 1::2]; c = img[1::2, 0::2]; d = img[1::2, 1::2]
        return (((a + b) + (c + d)) * F32(0.25)).astype(F32)

    def tab(ssz, dsz, clamp=True):
        scale = 1.0 / (dsz / ssz)
        ofs, a0, a1, lim = [], [], [], dsz
        for dd in range(dsz):
            fx = F32((dd + 0.5) * scale - 0.5)
            sx = int(math.floor(fx))
            fx = F32(fx - F32(sx))
            if clamp and sx < 0:
                fx, sx = F32(0), 0
            if clamp and sx + 1 >= ssz:
                lim = min(lim, dd)
                if sx >= ssz - 1:
                    fx, sx = F32(0), ssz - 1
            ofs.append(sx); a0.append(F32(1) - fx); a1.append(fx)
        return np.array(ofs), np.array(a0, F32), np.array(a1, F32), lim
    xo, xa0, xa1, xl = tab(sw, w)
    yo, ya0, ya1, _ = tab(sh, h, clamp=False)  # rows clipped below, weights keep fy
    xo1 = np.minimum(xo + 1, sw - 1)
    rows = img[:, xo] * xa0 + np.where(np.arange(w) < xl, img[:, xo1] * xa1, F32(0))
    r0 = rows[np.clip(yo, 0, sh - 1)]
    r1 = rows[np.clip(yo + 1, 0, sh - 1)]
    return (r0 * ya0[:, None] + r1 * ya1[:, None]).astype(F32)


def resize_nearest(m, w, h):
    sh, sw = m.shape[:2]
    if sw == w and sh == h:
        return m
    ifx, ify = 1.0 / (w / sw), 1.0 / (h / sh)
    xs = np.minimum(np.floor(np.arange(w) * ifx).astype(int), sw - 1)
    ys = np.minimum(np.floor(np.arange(h) * ify).astype(int), sh - 1)
    return m[ys][:, xs].copy()


def read_pairs(folder):
    lines = open(os.path.join(folder, "pair.txt")).read().splitlines()
    n = int(lines[0].split()[0])
    out = []
    for i in range(n):
        ref = int(lines[1 + 2 * i].split()[0])
        tok = lines[2 + 2 * i].split()
        srcs = [int(tok[1 + 2 * k]) for k in range(int(tok[0])) if float(tok[2 + 2 * k]) > 0]
        out.append((ref, srcs))
    return out


def run_schedule(folder, run_fn, seed_base=24301, ordering="sequential", use_sa=True, use_impetus=True,
                 dataset="ETH3D"):
    """Drive the whole reference schedule; returns {view: dict(depth, normal, weak, conf)} of the
    last pass. run_fn(arrays) -> A.Outputs (HIP engine or oracle)."""
    from PIL import Image
    problems = read_pairs(folder)
    ext = ".png"
    imgs = {ref: np.asarray(Image.open(os.path.join(folder, "images", f"{ref:08d}{ext}")), F32)
            for ref, _ in problems}
    cams = {ref: read_cam(os.path.join(folder, "cams", f"{ref:08d}_cam.txt")) for ref, _ in problems}
    H0, W0 = next(iter(imgs.values())).shape
    max_size, round_num = max(W0, H0), 1
    while max_size > 800:
        max_size //= 2
        round_num += 1
    geom_factor = 0.05 if dataset in ("TaT_a", "TaT_i") else 0.2
    store = {}  # view -> outputs of its latest pass
    masks = os.path.join(folder, "sa_masks")
    iteration = 0

    def one_pass(i, state, use_apd, geom, peak):
        nonlocal store
        snapshot = dict(store)
        for ref, srcs in problems:
            src_store = snapshot if ordering == "jacobi" else store
            ids = [ref] + srcs
            scale = 2 ** (round_num - 1 - i)
            cl = []
            images = []
            for k in ids:
                cam = dict(cams[k])
                img = imgs[k]
                h, w = img.shape
                if scale != 1:
                    factor = F32(1.0) / F32(scale)
                    nc, nr = int(round(float(F32(w) * factor))), int(round(float(F32(h) * factor)))
                    sx, sy = F32(nc) / F32(w), F32(nr) / F32(h)
                    img = resize_linear(img, nc, nr)
                    K = cam["K"].copy()
                    K[0] *= sx; K[2] *= sx; K[4] *= sy; K[5] *= sy
                    cam["K"] = K
                h, w = img.shape
                cam["width"], cam["height"] = w, h
                cl.append(cam)
                images.append(img)
            h, w = images[0].shape
            dmin = float(F32(cl[0]["depth_min"]) * F32(0.6))
            dmax = float(F32(cl[0]["depth_max"]) * F32(1.2))
            p = A.default_params(len(ids), dmin, dmax, state=state, use_APD=int(use_apd),
                                 geom_consistency=int(geom), weak_peak_radius=peak, use_sa=int(use_sa),
                                 use_impetus=int(use_impetus), geom_factor=geom_factor)
            if use_apd:
                p.ransac_threshold = float(F32(0.01 - i * 0.00125))
                p.rotate_time = min(int(2 ** i), 4)
            arr = A.ProblemArrays(w, h, images, cl, p, seed=seed_base ^ (iteration << 32) ^ ref)
            own = store.get(ref)
            if geom or use_apd:
                arr.depths = [resize_nearest(own["depth"], w, h)] + \
                             [resize_nearest(src_store[s]["depth"], w, h) for s in srcs]
            if use_apd:
                arr.weak_info = resize_nearest(own["weak"], w, h)
                arr.confidence = resize_nearest(own["conf"], w, h)
                if use_sa and os.path.isdir(masks):
                    arr.sa_mask = resize_nearest(synth.read_bin_mat(os.path.join(masks, f"{ref:08d}.bin")), w, h)
            if state != A.FIRST_INIT:
                d = resize_nearest(own["depth"], w, h)
                n = resize_nearest(own["normal"], w, h)
                arr.init_planes = np.concatenate([n, d[..., None]], -1).astype(F32)
            out = run_fn(arr)
            d = out.planes[..., 3].copy()
            wk = out.weak_info.copy()
            bad = (d < F32(dmin)) | (d > F32(dmax))
            d[bad] = 0
            wk[bad] = A.UNKNOWN
            conf = out.confidence.copy() if (geom or use_apd) else np.ones((h, w), np.uint8)
            store[ref] = dict(depth=d, normal=out.planes[..., :3].copy(), weak=wk, conf=conf)

    for i in range(round_num):
        one_pass(i, A.FIRST_INIT if i == 0 else A.REFINE_INIT, i > 0, False, 6)
        iteration += 1
        for j in range(3):
            one_pass(i, A.REFINE_ITER, i > 0, True, max(4 - 2 * j, 2))
            iteration += 1
    return store
