"""Save / load parity fixtures (tests/golden/*.npz): one apd_problem's inputs and the oracle's outputs.

A fixture is data only — inputs (images, cameras, params, priors, masks, seed) and the expected
outputs — loaded with numpy's default allow_pickle=False. tests/golden/make_golden.py writes them.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

import apd_abi as A

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CAM_FIELDS = ("K", "R", "t", "c", "height", "width", "depth_min", "depth_max", "interval", "depth_num")
OUT_FIELDS = ("planes", "costs", "weak_info", "confidence", "selected_views", "view_weights")


def save(path: str, arr: A.ProblemArrays, out: A.Outputs) -> None:
    d = {"width": np.int32(arr.width), "height": np.int32(arr.height), "seed": np.uint64(arr.seed)}
    imgs = np.stack([np.asarray(i, np.float32) for i in arr.images])
    if np.array_equal(imgs, np.round(imgs)) and imgs.min() >= 0 and imgs.max() <= 255:
        d["images_u8"] = imgs.astype(np.uint8)
    else:
        d["images_f32"] = imgs
    for f in CAM_FIELDS:
        d["cam_" + f] = np.array([np.asarray(c[f]) for c in arr.cameras])
    for name, _ in A.ApdParams._fields_:
        d["param_" + name] = np.array(getattr(arr.params, name))
    if arr.depths is not None:
        d["depths"] = np.stack([np.asarray(x, np.float32) for x in arr.depths])
    for f in ("init_planes", "weak_info", "confidence", "sa_mask"):
        v = getattr(arr, f)
        if v is not None:
            d["in_" + f] = np.asarray(v)
    for f in OUT_FIELDS:
        d["out_" + f] = getattr(out, f)
    wc = int(out.weak_count[0])
    d["out_weak_count"] = np.int32(wc)
    d["out_anchors"] = out.anchors[:wc].copy()
    np.savez_compressed(path, **d)


def load(path: str):
    z = np.load(path)  # allow_pickle=False (numpy default): data only
    imgs = z["images_u8"].astype(np.float32) if "images_u8" in z else z["images_f32"]
    n = imgs.shape[0]
    cams = []
    for i in range(n):
        c = {}
        for f in CAM_FIELDS:
            v = z["cam_" + f][i]
            c[f] = v if v.ndim else v.item()
        cams.append(c)
    params = A.ApdParams()
    for name, _ in A.ApdParams._fields_:
        setattr(params, name, z["param_" + name].item())
    arr = A.ProblemArrays(width=int(z["width"]), height=int(z["height"]), images=list(imgs), cameras=cams,
                          params=params, seed=int(z["seed"]))
    if "depths" in z:
        arr.depths = list(z["depths"])
    for f in ("init_planes", "weak_info", "confidence", "sa_mask"):
        if "in_" + f in z:
            setattr(arr, f, z["in_" + f])
    expected = {f: z["out_" + f] for f in OUT_FIELDS}
    expected["weak_count"] = int(z["out_weak_count"])
    expected["anchors"] = z["out_anchors"]
    return arr, expected


def fixtures():
    return sorted(os.path.join(GOLDEN_DIR, f) for f in os.listdir(GOLDEN_DIR) if f.endswith(".npz"))


def diff(expected: dict, got: A.Outputs) -> dict:
    """{field: differing elements}, bit-level (NaN == NaN)."""
    res = {}
    for f in OUT_FIELDS:
        x, y = expected[f], getattr(got, f)
        if x.dtype.kind == "f":
            same = (x.view(np.uint32) == y.view(np.uint32)) | (np.isnan(x) & np.isnan(y))
        else:
            same = x == y
        res[f] = int((~same).sum())
    wc = expected["weak_count"]
    res["weak_count"] = int(int(got.weak_count[0]) != wc)
    res["anchors"] = int((expected["anchors"] != got.anchors[:wc]).sum()) if wc else 0
    return res
