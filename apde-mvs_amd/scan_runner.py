"""View-sharded multi-GPU scan runner: one process per GPU, torch.distributed over RCCL.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29500 \
        apde-mvs_amd/scan_runner.py --dense_folder SCAN [--dataset ETH3D] [--seed 24301]

Runs the reference's whole depth schedule (main.cpp:290-367) over an MVSNet scan with the views of
every pass spread over the ranks. Within a pass a view depends on the other views only through their
state of the previous pass (depth maps for geometric consistency / APD priors, APD.cpp:592-610, plus
its own normals / pixel states / confidence), so the pass is Jacobi-ordered and its views are
independent: the ranks take them from a dynamic queue (an atomic counter on the rendezvous store),
longest first by the views' measured times in the previous pass -- per-view cost follows the WEAK
fraction -- and the pass ends with ONE collective, an all-gather of the new view
states, after which every rank holds every view's state. Results equal the `apd` binary with
--ordering jacobi and do not depend on the number of ranks or on which rank took which view. Rank 0
writes APD/<id>/{depths,normals,weak,confidence}.bin.

On GPUs the whole scan state stays in HBM: each round's resized images are uploaded once, the view
states live in torch tensors on the rank's device, libapd_hip.so reads its inputs from and writes
its outputs to them (device pointers through the C ABI), the INTER_NEAREST prior resizes are index
gathers on the device, and the all-gather runs device to device over RCCL (xGMI).

Host decoding and resizing go through the same C++ host library as the `apd` binary
(host/build/libapdhost.so); the PatchMatch itself is libapd_hip.so via apd_abi.Engine.
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys
import time
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
        A.torch_runtime_first()  # libapdhost.so links libapd_hip.so
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


def nearest_index(sw: int, sh: int, dw: int, dh: int):
    """Source rows / columns of cv::resize INTER_NEAREST from sw x sh to dw x dh, in the host library's
    arithmetic (host/image.cpp resize_nearest: floor(x * (1 / (dw / sw))) in double, clamped), so a
    gather with them equals the C++ resize element for element."""
    ifx, ify = 1.0 / (dw / sw), 1.0 / (dh / sh)
    xo = np.minimum(np.floor(np.arange(dw, dtype=np.float64) * ifx).astype(np.int64), sw - 1)
    yo = np.minimum(np.floor(np.arange(dh, dtype=np.float64) * ify).astype(np.int64), sh - 1)
    return yo, xo


class Exchange:
    """The per-pass step across ranks (torch.distributed): a dynamic view queue on the rendezvous
    store, and one all-gather of the new per-view state."""

    def __init__(self, world: int, rank: int, device: Optional[str]):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.world, self.rank, self.device = torch, dist, world, rank, device
        self.store = dist.distributed_c10d._get_default_store()

    def next_index(self, key: str) -> int:
        """Dynamic work queue: every rank draws the next position of the pass's view order from one
        atomic counter (TCPStore add), so a rank that finishes early takes more views."""
        return int(self.store.add(key, 1)) - 1

    def all_gather_state(self, mine: Dict[int, "object"], meta: Dict[int, float], h: int, w: int):
        """Every rank's new view states to every rank, on the device with RCCL when the ranks run on GPUs
        (no host round trip), plus the views' measured times for the next pass's queue order. On the
        wire a state is WIRE_BYTES_PER_PX = 18 B/px (wire_pack: depth + normal xyz as f32, pixel state
        + confidence as u8) instead of the [6, h, w] f32 it is held as (24 B/px)."""
        torch, dist = self.torch, self.dist
        ids = sorted(mine)
        lists = [None] * self.world
        dist.all_gather_object(lists, [(v, meta[v]) for v in ids])
        kmax = max(1, max(len(l) for l in lists))
        dev = self.device or "cpu"
        buf = torch.zeros((kmax, wire_bytes(h, w)), dtype=torch.uint8, device=dev)
        for k, v in enumerate(ids):
            buf[k] = wire_pack(mine[v])
        outs = [torch.empty_like(buf) for _ in range(self.world)]
        dist.all_gather(outs, buf)
        states, times = {}, {}
        for r in range(self.world):
            for k, (v, t) in enumerate(lists[r]):
                states[v] = wire_unpack(outs[r][k], h, w)
                times[v] = t
        return states, times

    def barrier(self):
        self.dist.barrier()


def _pack(depth, normal, weak, conf):
    import torch
    return torch.cat([depth[None], normal.permute(2, 0, 1), weak[None].float(), conf[None].float()], 0)


WIRE_BYTES_PER_PX = 4 * 4 + 2  # depth + normal xyz (f32), pixel state + confidence (u8)


def wire_bytes(h: int, w: int) -> int:
    """Bytes of one packed state, padded to 16 so that every state of a [k, wire_bytes] buffer starts
    4-byte aligned (its f32 planes are viewed in place)."""
    return (WIRE_BYTES_PER_PX * h * w + 15) // 16 * 16


def wire_pack(state):
    """A [6, h, w] f32 view state as the exchange's flat u8 buffer: the four f32 planes' bytes, then
    the pixel state and confidence planes as u8 (they hold small integers: exact both ways)."""
    import torch
    h, w = state.shape[-2], state.shape[-1]
    out = torch.zeros(wire_bytes(h, w), dtype=torch.uint8, device=state.device)
    n = 16 * h * w
    out[:n] = state[:4].contiguous().view(torch.uint8).reshape(-1)
    out[n:n + 2 * h * w] = state[4:6].to(torch.uint8).reshape(-1)
    return out


def wire_unpack(buf, h: int, w: int):
    """Inverse of wire_pack: the [6, h, w] f32 view state, bit-identical to the packed one."""
    import torch
    n = 4 * h * w
    f = buf[:4 * n].view(torch.float32).reshape(4, h, w)
    u = buf[4 * n:4 * n + 2 * h * w].reshape(2, h, w).float()
    return torch.cat([f, u], 0)


def run_scan(folder: str, run_fn: Callable, rank: int = 0, world: int = 1, exchange: Optional[Exchange] = None,
             dataset: str = "ETH3D", use_sa: bool = True, use_impetus: bool = True, seed: int = 24301,
             host: Optional[HostLib] = None, write: bool = True, device: Optional[str] = None):
    """The schedule of main.cpp:290-367 with Jacobi passes. Within a pass the ranks take views from a
    dynamic queue in longest-first order (the views' measured times in the previous pass: their cost
    follows the WEAK fraction), and the pass ends with one all-gather of the new states. Per round
    each image is decoded once and resized once (C++ host library), and -- with `device` -- kept on
    the GPU with every view's state, so problems pass device pointers to libapd_hip.so and nothing
    but the all-gather moves between passes. run_fn(ProblemArrays) -> outputs with planes, weak_info,
    confidence (numpy, or torch tensors on `device`). Returns {view: state tensor [6, h, w]} (every
    view on every rank)."""
    import torch
    host = host or HostLib()
    problems = read_pairs(folder)
    order = [p[0] for p in problems]
    prob = {p[0]: p for p in problems}
    ext = {p[0]: p[2] for p in problems}
    e0 = problems[0][2]
    dev = torch.device(device) if device else torch.device("cpu")
    needed = set(order)
    for _, srcs, _ in problems:
        needed.update(srcs)
    gray, cams = {}, {}
    for v in sorted(needed):  # decoded once per run (the apd binary's ImageCache)
        gray[v] = host.read_gray(os.path.join(folder, "images", f"{v:08d}{ext.get(v, e0)}")).astype(F32)
        cams[v] = host.read_camera(os.path.join(folder, "cams", f"{v:08d}_cam.txt"))
    H0, W0 = gray[order[0]].shape
    max_size, round_num = max(W0, H0), 1
    while max_size > 800:
        max_size //= 2
        round_num += 1
    geom_factor = 0.05 if dataset in ("TaT_a", "TaT_i") else 0.2
    masks = os.path.join(folder, "sa_masks")
    states: Dict[int, "torch.Tensor"] = {}  # every view: [6, h, w] of the previous pass
    times: Dict[int, float] = {}
    iteration = 0
    round_imgs: Dict[int, "torch.Tensor"] = {}
    round_cams: Dict[int, dict] = {}
    round_scale = [None]

    def load_round(scale):
        """Images and scaled cameras of one round: resized once per view (APD.cpp:562-590) and, with
        a device, uploaded once for all of the round's passes."""
        if round_scale[0] == scale:
            return
        round_imgs.clear()
        round_cams.clear()
        for v, img in gray.items():
            cam = dict(cams[v])
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
            round_cams[v] = cam
            round_imgs[v] = torch.from_numpy(np.ascontiguousarray(img)).to(dev)
        round_scale[0] = scale

    def fit(t, h, w):
        """INTER_NEAREST resize of a [.., h0, w0] tensor (priors, APD.cpp:592-672) as an index gather."""
        h0, w0 = t.shape[-2], t.shape[-1]
        if (h0, w0) == (h, w):
            return t
        yo, xo = nearest_index(w0, h0, w, h)
        yo, xo = torch.from_numpy(yo).to(t.device), torch.from_numpy(xo).to(t.device)
        return t.index_select(-2, yo).index_select(-1, xo)

    def one_pass(i, pstate, use_apd, geom, peak):
        nonlocal states, times
        scale = 2 ** (round_num - 1 - i)
        load_round(scale)
        h, w = round_imgs[order[0]].shape
        # longest first: the previous pass's measured times (ties and the first pass: pair.txt order)
        queue = sorted(order, key=lambda v: (-times.get(v, 0.0), order.index(v)))
        mine, meta = {}, {}
        key = f"apd_queue/{iteration}"
        k = exchange.next_index(key) if exchange else 0
        while k < len(queue):
            ref = queue[k]
            _, srcs, _ = prob[ref]
            ids = [ref] + srcs
            cl = [round_cams[v] for v in ids]
            dmin = float(F32(cl[0]["depth_min"]) * F32(0.6))
            dmax = float(F32(cl[0]["depth_max"]) * F32(1.2))
            p = A.default_params(len(ids), dmin, dmax, state=pstate, use_APD=int(use_apd),
                                 geom_consistency=int(geom), weak_peak_radius=peak, use_sa=int(use_sa),
                                 use_impetus=int(use_impetus), geom_factor=geom_factor)
            if use_apd:
                p.ransac_threshold = float(F32(0.01 - i * 0.00125))
                p.rotate_time = min(int(2 ** i), 4)
            arr = A.ProblemArrays(w, h, [round_imgs[v] for v in ids], cl, p, seed=seed ^ (iteration << 32) ^ ref)
            own = fit(states[ref], h, w) if ref in states else None
            if geom or use_apd:
                arr.depths = [fit(states[v][0], h, w).contiguous() for v in ids]
            if use_apd:
                arr.weak_info = own[4].to(torch.uint8).contiguous()
                arr.confidence = own[5].to(torch.uint8).contiguous()
                if use_sa and os.path.isdir(masks):
                    sa = torch.from_numpy(read_bin_mat(os.path.join(masks, f"{ref:08d}.bin"))).to(dev)
                    arr.sa_mask = fit(sa, h, w).contiguous()
            if pstate != A.FIRST_INIT:
                arr.init_planes = torch.cat([own[1:4].permute(1, 2, 0), own[0][..., None]], -1).contiguous()
            t0 = time.perf_counter()
            out = run_fn(arr)
            el = time.perf_counter() - t0
            planes = torch.as_tensor(out.planes, device=dev)
            d = planes[..., 3].clone()
            wk = torch.as_tensor(out.weak_info, device=dev).clone()
            bad = (d < F32(dmin)) | (d > F32(dmax))  # ProcessProblem epilogue (main.cpp:168-178)
            d[bad] = 0
            wk[bad] = A.UNKNOWN
            conf = torch.as_tensor(out.confidence, device=dev) if (geom or use_apd) else \
                torch.ones((h, w), dtype=torch.uint8, device=dev)
            mine[ref] = _pack(d, planes[..., :3], wk, conf)
            meta[ref] = el
            k = exchange.next_index(key) if exchange else k + 1
        # the exchange step: every rank gets every view's new state
        if exchange:
            states, times = exchange.all_gather_state(mine, meta, h, w)
        else:
            states, times = mine, meta

    for i in range(round_num):
        one_pass(i, A.FIRST_INIT if i == 0 else A.REFINE_INIT, i > 0, False, 6)
        iteration += 1
        for j in range(3):
            one_pass(i, A.REFINE_ITER, i > 0, True, max(4 - 2 * j, 2))
            iteration += 1
    if write and rank == 0:
        for v in order:
            st = states[v].cpu()
            d = os.path.join(folder, "APD", f"{v:08d}")
            os.makedirs(d, exist_ok=True)
            write_bin_mat(os.path.join(d, "depths.bin"), st[0].numpy().copy())
            write_bin_mat(os.path.join(d, "normals.bin"), st[1:4].permute(1, 2, 0).contiguous().numpy())
            write_bin_mat(os.path.join(d, "weak.bin"), st[4].numpy().astype(np.uint8))
            write_bin_mat(os.path.join(d, "confidence.bin"), st[5].numpy().astype(np.uint8))
    if exchange:
        exchange.barrier()  # every view written before any rank reports completion (fusion reads all)
    return states


def hip_run_fn(device: int, on_device: bool = False) -> Callable:
    """The HIP engine as run_fn; with on_device the outputs stay in HBM as torch tensors (inputs may be
    torch tensors on the same device: apd_set_problem / apd_get_results take device pointers)."""
    eng = A.Engine(device)

    def fn(arr):
        eng.set_problem(arr)
        eng.run()
        if on_device:
            return eng.results_device(arr.width, arr.height, f"cuda:{device}")
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
    on_device = torch.cuda.is_available()
    # one GPU per rank; APD_SCAN_DEVICES=n maps the ranks onto n devices (rank r -> device r mod n: a test
    # hook that runs several ranks on one GPU)
    ndev = int(os.environ.get("APD_SCAN_DEVICES", "0")) or (torch.cuda.device_count() if on_device else 1)
    dev_idx = local % max(1, ndev)
    if world > 1:
        # nccl == RCCL on ROCm; APD_SCAN_BACKEND=gloo exchanges the device tensors through gloo (test hook:
        # RCCL refuses two ranks on one GPU)
        backend = os.environ.get("APD_SCAN_BACKEND") or ("nccl" if on_device else "gloo")
        if on_device:
            torch.cuda.set_device(dev_idx)
        dist.init_process_group(backend)
        exchange = Exchange(world, rank, f"cuda:{dev_idx}" if on_device else None)
    run_fn = hip_run_fn(dev_idx, on_device)
    run_scan(args.dense_folder, run_fn, rank, world, exchange, dataset=args.dataset,
             use_sa=args.use_sa.lower() in ("1", "true", "yes", "on"),
             use_impetus=args.use_impetus.lower() in ("1", "true", "yes", "on"), seed=args.seed,
             device=f"cuda:{dev_idx}" if on_device else None)
    if exchange:
        dist.destroy_process_group()
    if rank == 0:
        print(f"scan done: {args.dense_folder} ({world} ranks)")


if __name__ == "__main__":
    main()
