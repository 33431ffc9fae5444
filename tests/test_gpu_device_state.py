"""GPU: the device-resident view-state functions of the C ABI (include/apd_hip.h).

* apd_device_resize_nearest == cv::resize INTER_NEAREST as the host restates it (host/image.cpp
  resize_nearest; tests/host_schedule.py resize_nearest, which test_gpu_cli ties to the binary),
  for every element size a prior has (u8 weak/conf/SA masks, f32 depth, f32x3 normals, f32x4
  planes) and the size pairs of the schedule (x2 up from a half-res round with odd sizes, identity,
  down). Bit-exact: it is an index gather.
* apd_result_device == the host epilogue (main.cpp:168-178 via apd_epilogue) of the same run:
  depth (0 outside [depth_min, depth_max], NaN kept) and (normal, depth) planes.
"""
import zlib

import numpy as np
import pytest

import apd_abi as A
import cases
import host_schedule as HS
import oracle_lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    lib = A.load_library()
    if lib.apd_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    eng = A.Engine(0, lib)
    yield eng
    eng.close()


SIZES = [((500, 375), (1000, 750)),     # a 2-round scan's half-res -> full-res
         ((503, 377), (1006, 754)),     # odd sizes: round(src / 2) then x2 is not the full size
         ((756, 504), (1512, 1008)),
         ((1000, 750), (1000, 750)),    # same size: still a gather (the ABI does not special-case it)
         ((1000, 750), (333, 251))]     # down


@pytest.mark.parametrize("src,dst", SIZES, ids=lambda s: f"{s[0]}x{s[1]}")
@pytest.mark.parametrize("kind", ["u8", "f32", "f32x3", "f32x4"])
def test_resize_nearest_equals_host(engine, src, dst, kind):
    import torch
    rng = np.random.default_rng(zlib.crc32(repr((src, dst, kind)).encode()))
    (sw, sh), (dw, dh) = src, dst
    if kind == "u8":
        m = rng.integers(0, 255, (sh, sw), dtype=np.uint8)
    else:
        c = {"f32": 1, "f32x3": 3, "f32x4": 4}[kind]
        m = rng.standard_normal((sh, sw, c) if c > 1 else (sh, sw)).astype(np.float32)
        m.reshape(-1)[::97] = np.nan  # a gather moves NaN payloads unchanged
    got = engine.resize_nearest_device(torch.from_numpy(m).to("cuda:0"), dw, dh).cpu().numpy()
    exp = HS.resize_nearest(m, dw, dh)
    assert got.shape == exp.shape
    assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(exp).view(np.uint8))


@pytest.mark.parametrize("name", ["refine_iter_apd_geom_sa", "first_n4"])
def test_result_device_equals_host_epilogue(engine, name):
    o = oracle_lib.load()
    arr = cases.make_case(name, lambda a: oracle_lib.run(o, a))
    engine.set_problem(arr)
    engine.run()
    W, H = arr.width, arr.height
    out = engine.results(A.Outputs(W, H, len(arr.images) - 1, max_weak=W * H))
    depth_d, planes_d = engine.result_device(W, H, "cuda:0")
    planes = np.ascontiguousarray(out.planes, np.float32).reshape(H, W, 4)
    depth = np.zeros((H, W), np.float32)
    normal = np.zeros((H, W, 3), np.float32)
    dmin, dmax = arr.params.depth_min, arr.params.depth_max
    st = engine.lib.apd_epilogue(W, H, A._ptr(planes, A.C.c_float), dmin, dmax, A._ptr(depth, A.C.c_float),
                                 A._ptr(normal, A.C.c_float), None)
    assert st == 0
    got_d = depth_d.cpu().numpy()
    got_p = planes_d.cpu().numpy()
    assert np.array_equal(got_d.view(np.uint32), depth.view(np.uint32))
    assert np.array_equal(got_p[..., :3].view(np.uint32), normal.view(np.uint32))
    assert np.array_equal(got_p[..., 3].view(np.uint32), depth.view(np.uint32))
