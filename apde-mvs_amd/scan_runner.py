"""View-sharded multi-GPU scan runner: one process per GPU, torch.distributed over RCCL.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29500 \
        apde-mvs_amd/scan_runner.py --dense_folder SCAN [--dataset ETH3D] [--seed 24301]

Runs the reference's whole depth schedule (main.cpp:290-367) over an MVSNet scan with the views of
every pass sharded across ranks (rank r owns views r, r+W, ...). Within a pass a view depends on the
other views only through their depth maps of the previous pass (geometric consistency / APD priors,
APD.cpp:592-610), so the pass is Jacobi-ordered: every rank processes its views against the
previous pass's maps, then ONE collective per pass -- an all-gather of the new depth maps, the only
cross-view data -- gives every rank the inputs of the next pass. Each view's own normal / weak /
confidence state stays on its owner. Results equal the `apd` binary with --ordering jacobi and are
independent of the number of ranks. Owners write APD/<id>/{depths,normals,weak,confidence}.bin.

Host decoding and resizing go through the same C++ host library as the `apd` binary
(host/build/libapdhost.so); the PatchMatch itself is libapd_hip.so via apd_abi.Engine.
"""
from __future__ import annotations

import argparse
import ctypes as C
import math
import os
import sys
from typing import Callable, Dict, List, Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)
import apd_abi as A  # noqa: E402

F32 = np.float32
HOSTLIB_PATH = os.path.join(HERE, "host", "build", "libapdhost.so")


class HostLib:
    """ctypes view of host/build/libapdhost.so (image decode, OpenCV-rule resize, cam.txt)."""

    def __init__(self, path: str = HOSTLIB_PATH):
        if not os.path.exists(path):
            raise A.ApdError(f"{path} not built: run `make -C apde-mvs_amd/host`")
        lib = C.CDLL(path)
        lib.apdhost_read_gray8.restype = C.c_long
        lib.apdhost_read_gray8.argtypes = [C.c_char_p, C.c_void_p, C.c_long, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        lib.apdhost_resize_linear_f32.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int]
        lib.apdhost_resize_nearest.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int]
        lib.apdhost_read_camera.restype = C.c_int
        lib.apdhost_read_camera.argtypes = [C.c_char_p, C.POINTER(A.ApdCamera)]
        self.lib = lib

    def read_gray(self, path: str) -> np.ndarray:
        w, h = C.c_int(), C.c_int()
        n = self.lib.apdhost_read_gray8(path.encode(), None, 0, C.byref(w), C.byref(h))
        if n <= 0:
            raise A.ApdError(f"cannot decode {path}")
        out = np.empty(n, np.uint8)
        self.lib.apdhost_read_gray8(path.encode(), out.ctypes.data, n, C.byref(w), C.byref(h))
        return out.reshape(h.value, w.value)

    def resize_linear(self, img: np.ndarray, w: int, h: int) -> np.ndarray:
        src = np.ascontiguousarray(img, F32)
        dst = np.empty((h, w), F32)
        self.lib.apdhost_resize_linear_f32(src.ctypes.data, src.shape[1], src.shape[0], dst.ctypes.data, w, h)
        return dst

    def resize_nearest(self, m: np.ndarray, w: int, h: int) -> np.ndarray:
        if m.shape[0] == h and m.shape[1] == w:
            return m
        src = np.ascontiguousarray(m)
        dst = np.empty((h, w) + m.shape[2:], m.dtype)
        self.lib.apdhost_resize_nearest(src.ctypes.data, m.shape[1], m.shape[0], dst.ctypes.data, w, h,
                                        src.itemsize * (int(np.prod(m.shape[2:])) if m.ndim > 2 else 1))
        return dst

    def read_camera(self, path: str) -> dict:
        cam = A.ApdCamera()
        if self.lib.apdhost_read_camera(path.encode(), C.byref(cam)) != 0:
            raise A.ApdError(f"cannot read {path}")
        return dict(K=np.array(cam.K[:], F32), R=np.array(cam.R[:], F32), t=np.array(cam.t[:], F32),
                    c=np.array(cam.c[:], F32), depth_min=F32(cam.depth_min), depth_max=F32(cam.depth_max),
                    interval=F32(cam.interval), depth_num=F32(cam.depth_num))


_CV = {(np.dtype(np.uint8), 1): 0, (np.dtype(np.int32), 1): 4, (np.dtype(np.float32), 1): 5,
       (np.dtype(np.float32), 3): 21}


def write_bin_mat(path: str, mat: np.ndarray) -> None:
    """WriteBinMat (APD.cpp:58-83)."""
    ch = 1 if mat.ndim == 2 else mat.shape[2]
    with open(path, "wb") as fh:
        np.array([1, mat.shape[0], mat.shape[1], _CV[(mat.dtype, ch)]], np.int32).tofile(fh)
        fh.write(np.ascontiguousarray(mat).tobytes())


def read_bin_mat(path: str) -> np.ndarray:
    """ReadBinMat (APD.cpp:18-56)."""
    with open(path, "rb") as fh:
        version, rows, cols, cvt = (int(v) for v in np.frombuffer(fh.read(16), np.int32))
        if version != 1:
            raise A.ApdError(f"bin-mat version {version}: {path}")
        dt, ch = {0: (np.uint8, 1), 4: (np.int32, 1), 5: (np.float32, 1), 21: (np.float32, 3)}[cvt]
        data = np.frombuffer(fh.read(), dt)
    return data.reshape((rows, cols) if ch == 1 else (rows, cols, ch)).copy()


def read_pairs(folder: str):
    """GenerateSampleList (main.cpp:44-102): (ref, [srcs with score > 0], image extension)."""
    lines = open(os.path.join(folder, "pair.txt")).read().splitlines()
    out = []
    for i in range(int(lines[0].split()[0])):
        ref = int(lines[1 + 2 * i].split()[0])
        tok = lines[2 + 2 * i].split()
        srcs = [int(tok[1 + 2 * k]) for k in range(int(tok[0])) if float(tok[2 + 2 * k]) > 0]
        ext = next((e for e in (".jpg", ".png", ".jpeg", ".JPG", ".PNG", ".JPEG")
                    if os.path.exists(os.path.join(folder, "images", f"{ref:08d}{e}"))), None)
        if ext is None:
            raise A.ApdError(f"can not find image: {ref:08d}")
        out.append((ref, srcs, ext))
    return out


class Exchange:
    """The per-pass collective: all-gather of the owners' new depth maps (torch.distributed)."""

    def __init__(self, world: int, rank: int, device: Optional[str]):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.world, self.rank, self.device = torch, dist, world, rank, device

    def all_gather_depths(self, owned: Dict[int, np.ndarray], order: List[int], h: int, w: int):
        torch, dist = self.torch, self.dist
        per = (len(order) + self.world - 1) // self.world
        mine = [v for v in order[self.rank::self.world]]
        buf = torch.zeros((per, h, w), dtype=torch.float32)
        for k, v in enumerate(mine):
            buf[k] = torch.from_numpy(owned[v])
        if self.device:
            buf = buf.to(self.device)
        outs = [torch.empty_like(buf) for _ in range(self.world)]
        dist.all_gather(outs, buf)
        res = {}
        for r in range(self.world):
            host = outs[r].cpu().numpy()
            for k, v in enumerate(order[r::self.world]):
                res[v] = host[k].copy()
        return res

    def barrier(self):
        self.dist.barrier()


def run_scan(folder: str, run_fn: Callable, rank: int = 0, world: int = 1, exchange: Optional[Exchange] = None,
             dataset: str = "ETH3D", use_sa: bool = True, use_impetus: bool = True, seed: int = 24301,
             host: Optional[HostLib] = None, write: bool = True):
    """The schedule of main.cpp:290-367 with Jacobi passes over the views owned by `rank`.
    run_fn(ProblemArrays) -> apd_abi.Outputs. Returns {view: state} for the owned views."""
    host = host or HostLib()
    problems = read_pairs(folder)
    order = [p[0] for p in problems]
    owned_ids = order[rank::world]
    imgs, cams = {}, {}
    needed = set(owned_ids)
    for ref, srcs, _ in problems:
        if ref in needed:
            needed.update(srcs)
    ext = {p[0]: p[2] for p in problems}
    e0 = problems[0][2]
    for v in sorted(needed):
        imgs[v] = host.read_gray(os.path.join(folder, "images", f"{v:08d}{ext.get(v, e0)}")).astype(F32)
        cams[v] = host.read_camera(os.path.join(folder, "cams", f"{v:08d}_cam.txt"))
    H0, W0 = imgs[owned_ids[0]].shape if owned_ids else next(iter(imgs.values())).shape
    max_size, round_num = max(W0, H0), 1
    while max_size > 800:
        max_size //= 2
        round_num += 1
    geom_factor = 0.05 if dataset in ("TaT_a", "TaT_i") else 0.2
    state: Dict[int, dict] = {}        # owned views: depth, normal, weak, conf
    depths: Dict[int, np.ndarray] = {}  # every view's depth of the previous pass
    masks = os.path.join(folder, "sa_masks")
    iteration = 0

    def one_pass(i, pstate, use_apd, geom, peak):
        nonlocal depths
        scale = 2 ** (round_num - 1 - i)
        w = h = None
        for ref, srcs, _ in problems:
            if ref not in owned_ids:
                continue
            ids = [ref] + srcs
            images, cl = [], []
            for k in ids:
                cam = dict(cams[k])
                img = imgs[k]
                ih, iw = img.shape
                if scale != 1:
                    factor = F32(1.0) / F32(scale)
                    nc, nr = int(round(float(F32(iw) * factor))), int(round(float(F32(ih) * factor)))
                    sx, sy = F32(nc) / F32(iw), F32(nr) / F32(ih)
                    img = host.resize_linear(img, nc, nr)
                    K = cam["K"].copy()
                    K[0] *= sx; K[2] *= sx; K[4] *= sy; K[5] *= sy
                    cam["K"] = K
                ih, iw = img.shape
                cam["width"], cam["height"] = iw, ih
                cl.append(cam)
                images.append(img)
            h, w = images[0].shape
            dmin = float(F32(cl[0]["depth_min"]) * F32(0.6))
            dmax = float(F32(cl[0]["depth_max"]) * F32(1.2))
            p = A.default_params(len(ids), dmin, dmax, state=pstate, use_APD=int(use_apd),
                                 geom_consistency=int(geom), weak_peak_radius=peak, use_sa=int(use_sa),
                                 use_impetus=int(use_impetus), geom_factor=geom_factor)
            if use_apd:
                p.ransac_threshold = float(F32(0.01 - i * 0.00125))
                p.rotate_time = min(int(2 ** i), 4)
            arr = A.ProblemArrays(w, h, images, cl, p, seed=seed ^ (iteration << 32) ^ ref)
            own = state.get(ref)
            if geom or use_apd:
                arr.depths = [host.resize_nearest(depths[v], w, h) for v in ids]
            if use_apd:
                arr.weak_info = host.resize_nearest(own["weak"], w, h)
                arr.confidence = host.resize_nearest(own["conf"], w, h)
                if use_sa and os.path.isdir(masks):
                    arr.sa_mask = host.resize_nearest(read_bin_mat(os.path.join(masks, f"{ref:08d}.bin")), w, h)
            if pstate != A.FIRST_INIT:
                d = host.resize_nearest(own["depth"], w, h)
                n = host.resize_nearest(own["normal"], w, h)
                arr.init_planes = np.concatenate([n, d[..., None]], -1).astype(F32)
            out = run_fn(arr)
            d = out.planes[..., 3].copy()
            wk = out.weak_info.copy()
            bad = (d < F32(dmin)) | (d > F32(dmax))  # ProcessProblem epilogue (main.cpp:168-178)
            d[bad] = 0
            wk[bad] = A.UNKNOWN
            conf = out.confidence.copy() if (geom or use_apd) else np.ones((h, w), np.uint8)
            state[ref] = dict(depth=d, normal=out.planes[..., :3].copy(), weak=wk, conf=conf)
        # the exchange step: every rank gets every view's new depth map
        if h is None:  # a rank without views still takes part in the collective
            h, w = (round(H0 / scale), round(W0 / scale))
        new = {v: state[v]["depth"] for v in owned_ids}
        depths = exchange.all_gather_depths(new, order, h, w) if exchange else dict(new)

    for i in range(round_num):
        one_pass(i, A.FIRST_INIT if i == 0 else A.REFINE_INIT, i > 0, False, 6)
        iteration += 1
        for j in range(3):
            one_pass(i, A.REFINE_ITER, i > 0, True, max(4 - 2 * j, 2))
            iteration += 1
    if write:
        for v in owned_ids:
            d = os.path.join(folder, "APD", f"{v:08d}")
            os.makedirs(d, exist_ok=True)
            write_bin_mat(os.path.join(d, "depths.bin"), state[v]["depth"])
            write_bin_mat(os.path.join(d, "normals.bin"), state[v]["normal"])
            write_bin_mat(os.path.join(d, "weak.bin"), state[v]["weak"])
            write_bin_mat(os.path.join(d, "confidence.bin"), state[v]["conf"])
    if exchange:
        exchange.barrier()  # every view written before any rank reports completion (fusion reads all)
    return state


def hip_run_fn(device: int) -> Callable:
    eng = A.Engine(device)

    def fn(arr):
        eng.set_problem(arr)
        eng.run()
        return eng.results(A.Outputs(arr.width, arr.height, len(arr.images) - 1))
    fn.engine = eng
    return fn


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--dense_folder", required=True)
    ap.add_argument("--dataset", default="ETH3D")
    ap.add_argument("--use_sa", default="true")
    ap.add_argument("--use_impetus", default="true")
    ap.add_argument("--seed", type=int, default=24301)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    exchange = None
    if world > 1:
        backend = "nccl" if torch.cuda.is_available() else "gloo"  # nccl == RCCL on ROCm
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend)
        exchange = Exchange(world, rank, f"cuda:{local}" if backend == "nccl" else None)
    run_fn = hip_run_fn(local)
    run_scan(args.dense_folder, run_fn, rank, world, exchange, dataset=args.dataset,
             use_sa=args.use_sa.lower() in ("1", "true", "yes", "on"),
             use_impetus=args.use_impetus.lower() in ("1", "true", "yes", "on"), seed=args.seed)
    if exchange:
        dist.destroy_process_group()
    if rank == 0:
        print(f"scan done: {args.dense_folder} ({world} ranks)")


if __name__ == "__main__":
    main()
