"""Known-answer tests for the APD half of the oracle (CPU only).

The HIP kernels are checked bit-for-bit against oracle/apd_oracle.c; these tests pin the oracle's APD
functions to answers derived independently of it -- hand-built inputs whose result follows from the
reference's text, or numpy restatements written from the reference lines cited per test:

* ComputeBilateralNCCNew's focal combination (APD.cu:431-446, 495-586): identical anchor windows give
  0.25 * c0 + 0.75 * c; an anchor projected out of the source image whose selected views hold the
  source gives a 2.0 entry of the softmax (and none without the bit);
* DepthToWeak's classification (APD.cu:2200-2249) on hand-built 61-sample curves, on random curves
  against a numpy restatement, and on the curves a real run exports (--export_curve) against its
  pixel states;
* ConfidenceCompute's counts (APD.cu:2282-2344) against a float64 numpy restatement;
* CheckerboardFilterStrong's 21-tap median (APD.cu:1711-1855), black then red, on integer depths;
* FindNearestStrongPoint (APD.cu:2434-2484) against a numpy brute force;
* GenAnchors + NeigbourUpdate (APD.cu:1857-2100) on hand-built STRONG maps with known directional
  points and coplanar / off-plane depths.
Each test also mutates one reference quirk in its restatement where that is meaningful and checks
that the oracle disagrees, so a test that cannot fail is caught.
"""
import ctypes as C

import numpy as np
import pytest

import apd_abi as A
import cases
import oracle_lib


@pytest.fixture(scope="module")
def lib():
    lib = oracle_lib.load()
    lib.oracle_classify_curve.restype = C.c_int
    lib.oracle_classify_curve.argtypes = [C.POINTER(C.c_float), C.c_int]
    lib.oracle_ncc_new.restype = C.c_float
    lib.oracle_ncc_new.argtypes = [C.POINTER(A.ApdProblem), C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float),
                                   C.POINTER(C.c_int16), C.POINTER(C.c_uint32)]
    lib.oracle_kat_stage.restype = C.c_int
    lib.oracle_kat_stage.argtypes = [C.POINTER(A.ApdProblem), C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    return lib


def ptr(a):
    return None if a is None else a.ctypes.data


# ------------------------------------------------------------------------------------------------
# DepthToWeak classification, APD.cu:2200-2249

def classify_np(pc, radius, strict_peak=True, single_thr=0.15):
    """numpy/float32 restatement of APD.cu:2200-2249 (quirk switches for the mutation checks)."""
    pc = np.asarray(pc, np.float32)
    peaks = []
    for i in range(2, 59):
        if (pc[i - 1] > pc[i] and pc[i + 1] > pc[i]) if strict_peak else (pc[i - 1] >= pc[i] and pc[i + 1] >= pc[i]):
            peaks.append(i)
    min_peak, min_cost = 0, np.float32(2.0)
    for i in peaks:
        if pc[i] < min_cost:
            min_peak, min_cost = i, pc[i]
    if abs(min_peak - 30) > radius or pc[min_peak] > np.float32(0.5):
        return A.WEAK
    if len(peaks) == 1:
        return A.STRONG if pc[min_peak] <= np.float32(single_thr) else A.WEAK
    var = np.float32(0.0)
    for i in peaks:
        if i != min_peak:
            d = np.float32(pc[i] - min_cost)
            var = np.float32(np.float64(d) * np.float64(d) + np.float64(var))  # exact on the 1/64 grid below
    var = np.float32(np.sqrt(var)) / np.float32(len(peaks) - 1)
    return A.STRONG if var > np.float32(0.2) else A.WEAK


def vee(centre, depth, slope=0.02, base=1.6):
    """A curve with one minimum `depth` at sample `centre`, rising by `slope` per sample."""
    i = np.arange(61)
    return np.minimum(base, depth + slope * np.abs(i - centre)).astype(np.float32)


def multi(minima, slope=0.05, base=1.6):
    i = np.arange(61)
    c = np.full(61, base, np.float32)
    for centre, depth in minima:
        c = np.minimum(c, depth + slope * np.abs(i - centre))
    return c.astype(np.float32)


def oracle_classify(lib, pc, radius):
    pc = np.ascontiguousarray(pc, np.float32)
    return lib.oracle_classify_curve(pc.ctypes.data_as(C.POINTER(C.c_float)), radius)


HAND_CURVES = [
    # (curve, weak_peak_radius, expected, why)
    (vee(30, 0.10), 6, A.STRONG, "single minimum 0.10 <= 0.15 at the centre"),
    (vee(30, 0.15), 6, A.STRONG, "single minimum exactly 0.15 (<=)"),
    (vee(30, 0.20), 6, A.WEAK, "single minimum 0.20 > 0.15"),
    (vee(30, 0.60), 6, A.WEAK, "lowest peak costs > 0.5"),
    (vee(34, 0.10), 4, A.STRONG, "minimum at centre + radius"),
    (vee(35, 0.10), 4, A.WEAK, "minimum at centre + radius + 1"),
    (vee(26, 0.10), 4, A.STRONG, "minimum at centre - radius"),
    (vee(1, 0.05), 6, A.WEAK, "minimum at sample 1 is not a peak (samples 2..58 only): no peak"),
    (np.linspace(1.5, 0.2, 61), 6, A.WEAK, "monotone: no peak, min_peak 0 is 30 away"),
    (multi([(30, 0.10), (45, 0.40)]), 6, A.STRONG, "two peaks, spread 0.30 > 0.2"),
    (multi([(30, 0.10), (45, 0.25)]), 6, A.WEAK, "two peaks, spread 0.15 <= 0.2"),
    (multi([(30, 0.10), (10, 0.40), (50, 0.40)]), 6, A.STRONG, "three peaks, sqrt(2 * 0.3^2) / 2 = 0.212"),
    (multi([(30, 0.10), (10, 0.35), (50, 0.35)]), 6, A.WEAK, "three peaks, sqrt(2 * 0.25^2) / 2 = 0.177"),
    (multi([(10, 0.10), (30, 0.12)]), 6, A.WEAK, "lowest peak 20 samples from the centre"),
]


@pytest.mark.parametrize("k", range(len(HAND_CURVES)), ids=[h[3] for h in HAND_CURVES])
def test_classify_hand_built_curves(lib, k):
    pc, radius, expected, _ = HAND_CURVES[k]
    assert classify_np(pc, radius) == expected
    assert oracle_classify(lib, pc, radius) == expected


def test_classify_plateau_is_not_a_peak(lib):
    pc = multi([(30, 0.10), (33, 0.12)])
    pc[31] = pc[30]  # flat bottom at 30/31: neither sample is strictly below both neighbours
    # the only peak is 33 (0.12 <= 0.15, 3 from the centre): STRONG
    assert oracle_classify(lib, pc, 6) == A.STRONG
    assert classify_np(pc, 6) == A.STRONG
    # mutation (peaks with >=): 30, 31 and 33 are peaks, spread 0.02 / 2 -> WEAK
    assert classify_np(pc, 6, strict_peak=False) == A.WEAK


def test_classify_random_curves_match_restatement(lib):
    rng = np.random.default_rng(7)
    mism = 0
    for t in range(4000):
        if t % 2:  # smooth curves around a random centre (peaks near the thresholds' scale)
            pc = multi([(int(rng.integers(2, 59)), rng.integers(0, 40) / 64.0) for _ in range(rng.integers(1, 4))],
                       slope=rng.integers(1, 8) / 64.0)
        else:
            pc = rng.integers(0, 129, 61) / 64.0
        pc = np.round(np.asarray(pc) * 64) / 64  # exact in fp32 and in the squared sums
        r = int(rng.choice([2, 4, 6]))
        mism += classify_np(pc, r) != oracle_classify(lib, pc, r)
    assert mism == 0


def band_decides_weak(pc, radius):
    """k_depth_to_weak_vm's inner-band verdict (DW_EARLY): no local minimum i with |i - 30| <= radius
    (and 2 <= i <= 58) costs <= 0.5, so the pixel is WEAK whatever its other samples are."""
    for i in range(max(2, 30 - radius), min(58, 30 + radius) + 1):
        if pc[i - 1] > pc[i] and pc[i + 1] > pc[i] and pc[i] <= 0.5:
            return False
    return True


def test_inner_band_rule_is_exact(lib):
    """The rule the GPU's DepthToWeak uses to skip the outer disparities of a pixel: whenever it says
    WEAK, the reference's classification of the full curve (APD.cu:2200-2249, the oracle) is WEAK --
    on random curves, on curves built around the band's edges, and whatever the outer samples hold
    (they are redrawn). The band [min(25, 29 - r), max(36, 32 + r)) holds every sample the rule reads."""
    rng = np.random.default_rng(11)
    decided = 0
    for t in range(6000):
        r = int(rng.choice([2, 4, 6]))
        if t % 3 == 0:
            pc = rng.integers(0, 129, 61) / 64.0
        elif t % 3 == 1:  # a minimum near the band's edge or just above the 0.5 limit
            c = 30 + int(rng.choice([-r - 1, -r, r, r + 1]))
            pc = multi([(c, rng.choice([0.25, 0.5, 33 / 64.0]))] +
                       [(int(rng.integers(2, 59)), rng.integers(0, 40) / 64.0) for _ in range(rng.integers(0, 3))],
                       slope=rng.integers(1, 8) / 64.0)
        else:
            pc = multi([(int(rng.integers(2, 59)), rng.integers(0, 40) / 64.0) for _ in range(rng.integers(1, 4))],
                       slope=rng.integers(1, 8) / 64.0)
        pc = np.round(np.asarray(pc, np.float64) * 64) / 64
        lo, hi = min(25, 29 - r), max(36, 32 + r)
        assert lo <= max(2, 30 - r) - 1 and min(58, 30 + r) + 1 < hi
        if not band_decides_weak(pc, r):
            continue
        decided += 1
        assert oracle_classify(lib, pc, r) == A.WEAK
        # the verdict does not depend on the samples outside the band
        pc2 = pc.copy()
        outer = np.r_[0:lo, hi:61]
        pc2[outer] = rng.integers(0, 129, outer.size) / 64.0
        assert oracle_classify(lib, pc2, r) == A.WEAK
    assert decided > 1000
    # control: a qualifying minimum at the band's edge (cost 0.5, |i - 30| = r) is not decided, and
    # the full curve can be STRONG
    pc = vee(30 + 4, 0.5)
    assert not band_decides_weak(pc, 4)
    pc = vee(30 + 4, 0.10)
    assert not band_decides_weak(pc, 4) and oracle_classify(lib, pc, 4) == A.STRONG
    # mutation control (a band rule with < 0.5 instead of <= 0.5 would be wrong): an inner minimum of
    # exactly 0.5 with a far peak 0.28 above it is STRONG by the spread test
    pc = multi([(30, 0.5), (10, 0.78)])
    assert oracle_classify(lib, pc, 4) == A.STRONG and not band_decides_weak(pc, 4)


def test_classify_matches_exported_curves():
    """--export_curve (APD.cu:2188-2198): every pixel DepthToWeak classified from a curve gets the
    state the numpy restatement gives that exported curve (FIRST_INIT: nothing changes the states
    after DepthToWeak)."""
    lib = oracle_lib.load()
    sc = cases.scene(96, 72, 4)
    arr = cases.base_problem(sc, 0)
    arr.export_reliable_curve = True
    out = oracle_lib.run(lib, arr, 8, want_curve=True)
    curves = out.reliable_curve.reshape(72, 96, 61)
    radius = arr.params.weak_peak_radius
    checked = 0
    for y in range(6, 66):
        for x in range(6, 90):
            if out.weak_info[y, x] == A.UNKNOWN:
                continue
            assert classify_np(curves[y, x], radius) == out.weak_info[y, x], (x, y)
            checked += 1
    assert checked > 3000
    assert (out.weak_info == A.STRONG).any() and (out.weak_info == A.WEAK).any()


# ------------------------------------------------------------------------------------------------
# NCC-New focal combination, APD.cu:431-446, 448-593

def _weak_problem(sc):
    arr = cases.base_problem(sc, 0)
    arr.params.use_APD = 1
    arr.params.state = A.REFINE_INIT
    arr.weak_info = np.full((sc.height, sc.width), A.WEAK, np.uint8)
    arr.depths = list(sc.gt_depth[:len(arr.images)])
    arr.init_planes = np.zeros((sc.height, sc.width, 4), np.float32)
    return arr


def _plane(lib, arr, px, py, depth):
    """A fronto-parallel reference-frame plane through (px, py) at `depth`."""
    cam = arr.build().cameras[0]
    n = np.array([0.0, 0.0, -1.0, 0.0], np.float32)
    w = lib.oracle_dist2origin(C.byref(cam), px, py, depth, n.ctypes.data_as(C.POINTER(C.c_float)))
    return np.array([0.0, 0.0, -1.0, w], np.float32)


def _fma32(a, b, c):
    return np.float32(np.float64(np.float32(a)) * np.float64(np.float32(b)) + np.float64(np.float32(c)))


def _project32(H9, x, y):
    """ComputeCorrespondingPoint (APD.cu:396-403) in the build's fp32 contract (nvcc's contracted
    multiply-adds and the fast-math X * rcp(Z), oracle header): the texel lookup rounds the position
    to 1/256, so the projection must round like the engine for the window values to agree."""
    X = _fma32(H9[1], y, _fma32(H9[0], x, H9[2]))
    Y = _fma32(H9[4], y, _fma32(H9[3], x, H9[5]))
    Z = _fma32(H9[7], y, _fma32(H9[6], x, H9[8]))
    iz = np.float32(1.0) / Z
    return float(np.float32(X * iz)), float(np.float32(Y * iz))


def _window_ncc(lib, arr, H9, ax, ay, radius, inc, src):
    """Restatement of one window of ComputeBilateralNCCNew (APD.cu:513-563): reference texels at
    integer positions (clamped), source texels bilinear at the projection (the KAT-pinned
    oracle_tex_bilinear), and the moments in fp32 as the reference accumulates them (weight 1, nvcc's
    contracted multiply-adds): the textureless windows a WEAK pixel sees have variances of ~1 on
    means of ~128, so the fp32 cancellation in E[r^2] - E[r]^2 is part of the reference's answer."""
    W, H = arr.width, arr.height
    ref = arr.images[0]
    img = np.ascontiguousarray(arr.images[src], np.float32)
    f32 = np.float32
    sr = srr = ss = sss = srs = wsum = f32(0.0)
    for i in range(-radius, radius + 1, inc):
        for j in range(-radius, radius + 1, inc):
            x, y = ax + i, ay + j
            r = f32(ref[min(max(y, 0), H - 1), min(max(x, 0), W - 1)])
            sx, sy = _project32(H9, x, y)
            v = f32(lib.oracle_tex_bilinear(img.ctypes.data_as(C.POINTER(C.c_float)), W, H, sx, sy))
            sr = f32(sr + r)
            srr = _fma32(r, r, srr)
            ss = f32(ss + v)
            sss = _fma32(v, v, sss)
            srs = _fma32(r, v, srs)
            wsum = f32(wsum + f32(1.0))
    inv = f32(1.0) / wsum
    sr, srr, ss, sss, srs = (f32(t * inv) for t in (sr, srr, ss, sss, srs))
    vr, vs = _fma32(-sr, sr, srr), _fma32(-ss, ss, sss)
    if vr < f32(1e-5) or vs < f32(1e-5):
        return 2.0
    cov = _fma32(-sr, ss, srs)
    return float(max(f32(0.0), min(f32(2.0), f32(f32(1.0) - f32(cov / f32(np.sqrt(f32(vr * vs))))))))


def _ncc_new(lib, arr, px, py, src, plane, anchors, sel=None):
    pb = arr.build()
    anc = np.ascontiguousarray(np.asarray(anchors, np.int16).reshape(9, 2))
    sel_a = None if sel is None else np.ascontiguousarray(sel, np.uint32)
    return lib.oracle_ncc_new(C.byref(pb), px, py, src, plane.ctypes.data_as(C.POINTER(C.c_float)),
                              anc.ctypes.data_as(C.POINTER(C.c_int16)),
                              None if sel_a is None else sel_a.ctypes.data_as(C.POINTER(C.c_uint32)))


def _homography(lib, arr, src, plane):
    H9 = np.zeros(9, np.float32)
    pb = arr.build()
    lib.oracle_homography(C.byref(pb), src, plane.ctypes.data_as(C.POINTER(C.c_float)),
                          H9.ctypes.data_as(C.POINTER(C.c_float)))
    return H9


def test_ncc_new_identical_anchor_windows(lib):
    """All 8 anchors at one pixel q: the softmax weights are exactly 1/8 each, so the focal cost is
    the anchor window's cost c and NCC-New = 0.25 * c0 + 0.75 * min(c, 2) (APD.cu:576-586), with c0
    the 6x6 centre window (== NCC-Old of the same plane) and c the 3x3 step-5 window at q."""
    sc = cases.scene(96, 72, 4)
    arr = _weak_problem(sc)
    px, py, q = 48, 36, (53, 33)
    for src in (1, 2):
        pl = _plane(lib, arr, px, py, float(sc.gt_depth[0][py, px]))
        got = _ncc_new(lib, arr, px, py, src, pl, [(px, py)] + [q] * 8)
        pb = arr.build()
        c0 = lib.oracle_ncc_old(C.byref(pb), px, py, src, pl.ctypes.data_as(C.POINTER(C.c_float)))
        H9 = _homography(lib, arr, src, pl)
        assert abs(c0 - _window_ncc(lib, arr, H9, px, py, 5, 2, src)) < 2e-5
        c = _window_ncc(lib, arr, H9, q[0], q[1], 5, 5, src)
        assert abs(got - (0.25 * c0 + 0.75 * min(c, 2.0))) < 2e-5, (src, got, c0, c)
        # mutation: the reference's 0.25/0.75 mix, not an equal one
        assert abs(got - 0.5 * (c0 + c)) > 1e-4 or abs(c0 - c) < 1e-4


def test_ncc_new_softmax_of_distinct_anchor_windows(lib):
    """Anchors at 8 different pixels: focal cost = sum softmax(c)_i c_i (APD.cu:431-446, 576-585)."""
    sc = cases.scene(96, 72, 4)
    arr = _weak_problem(sc)
    px, py, src = 40, 30, 1
    qs = [(44, 30), (36, 30), (40, 34), (40, 26), (45, 35), (35, 25), (45, 25), (35, 35)]
    pl = _plane(lib, arr, px, py, float(sc.gt_depth[0][py, px]))
    got = _ncc_new(lib, arr, px, py, src, pl, [(px, py)] + qs)
    H9 = _homography(lib, arr, src, pl)
    c0 = _window_ncc(lib, arr, H9, px, py, 5, 2, src)
    c = np.array([_window_ncc(lib, arr, H9, x, y, 5, 5, src) for x, y in qs])
    w = np.exp(c - c.max())
    w /= w.sum()
    focal = min(float((w * c).sum()), 2.0)
    assert abs(got - (0.25 * c0 + 0.75 * focal)) < 3e-5
    # mutation: a plain mean of the anchor costs instead of the softmax weighting
    if np.ptp(c) > 0.05:
        assert abs(got - (0.25 * c0 + 0.75 * c.mean())) > 1e-4


def test_ncc_new_out_of_frame_anchor(lib):
    """An anchor whose projection leaves the source image contributes a 2.0 entry iff its selected
    views contain the source (APD.cu:499-512); without the bit it is skipped. Anchor 0 (the pixel
    itself) out of frame makes the whole cost 2.0 (checked on the centre projection, APD.cu:472-475)."""
    sc = cases.scene(96, 72, 4)
    arr = _weak_problem(sc)
    px, py, src = 10, 36, 1
    pl = _plane(lib, arr, px, py, float(sc.gt_depth[0][py, px]))
    H9 = _homography(lib, arr, src, pl)
    # find a reference pixel left of the image whose projection is out of frame: use x = 0 rows and
    # pick the in-image anchor with the smallest projected x; if even x = 0 lands inside, shift the
    # plane far away so that the left border projects outside
    out_q = None
    for x in range(0, 96):
        for y in (5, 36, 66):
            X, Yv = _project32(H9, x, y)
            if not (0 <= X < 96 and 0 <= Yv < 72):
                out_q = (x, y)
                break
        if out_q:
            break
    if out_q is None:
        pytest.skip("no out-of-frame anchor for this scene/view")
    ins = [(14, 36), (10, 40), (14, 40), (10, 32), (14, 32), (12, 38), (12, 34)]
    anchors = [(px, py), out_q] + ins
    sel = np.zeros((72, 96), np.uint32)
    got_skip = _ncc_new(lib, arr, px, py, src, pl, anchors, sel)
    sel[out_q[1], out_q[0]] = 1 << (src - 1)
    got_two = _ncc_new(lib, arr, px, py, src, pl, anchors, sel)
    c0 = _window_ncc(lib, arr, H9, px, py, 5, 2, src)
    c = np.array([_window_ncc(lib, arr, H9, x, y, 5, 5, src) for x, y in ins])

    def mix(cs):
        w = np.exp(cs - cs.max())
        w /= w.sum()
        return 0.25 * c0 + 0.75 * min(float((w * cs).sum()), 2.0)

    assert abs(got_skip - mix(c)) < 3e-5
    assert abs(got_two - mix(np.concatenate([[2.0], c]))) < 3e-5
    assert abs(got_two - got_skip) > 1e-4


# ------------------------------------------------------------------------------------------------
# ConfidenceCompute, APD.cu:2282-2344

def _confidence_np(arr, planes, sel):
    """float64 restatement of ConfidenceCompute; returns (conf, margin) where margin flags pixels
    whose count depends on a comparison within float32 rounding of its threshold."""
    Hh, W = arr.height, arr.width
    cams = [arr.cameras[i] for i in range(len(arr.images))]
    K = [np.asarray(c["K"], np.float64).reshape(3, 3) for c in cams]
    R = [np.asarray(c["R"], np.float64).reshape(3, 3) for c in cams]
    t = [np.asarray(c["t"], np.float64) for c in cams]
    cc = [np.asarray(c["c"], np.float64) for c in cams]
    conf = np.zeros((Hh, W), np.int32)
    margin = np.zeros((Hh, W), bool)
    for y in range(Hh):
        for x in range(W):
            rd = float(planes[y, x, 3])
            if rd <= 0:
                continue
            P = np.array([rd * (x - K[0][0, 2]) / K[0][0, 0], rd * (y - K[0][1, 2]) / K[0][1, 1], rd])
            Xw = R[0].T @ P + cc[0]  # Get3DPointonWorld_cu: R^T (camera-frame point) + c
            n = 1
            for i in range(len(cams) - 1):
                if not (int(sel[y, x]) >> i) & 1:
                    continue
                s = i + 1
                tmp = R[s] @ Xw + t[s]
                d = K[s][2] @ tmp
                sx, sy = (K[s][0] @ tmp) / d, (K[s][1] @ tmp) / d
                ix = min(max(int(sx), 0), W - 1) if np.isfinite(sx) else 0
                iy = min(max(int(sy), 0), Hh - 1) if np.isfinite(sy) else 0
                if abs(sx - round(sx)) < 1e-3 or abs(sy - round(sy)) < 1e-3:
                    margin[y, x] = True
                sd = float(arr.depths[s][iy, ix])
                if sd <= 0:
                    continue
                n += 1
                Q = np.array([sd * (sx - K[s][0, 2]) / K[s][0, 0], sd * (sy - K[s][1, 2]) / K[s][1, 1], sd])
                Qw = R[s].T @ Q + cc[s]
                tmp = R[0] @ Qw + t[0]
                rdd = K[0][2] @ tmp
                bx, by = (K[0][0] @ tmp) / rdd, (K[0][1] @ tmp) / rdd
                e = np.hypot(x - bx, y - by)
                rel = abs(rd - rdd) / rd
                if abs(e - 2.0) < 1e-3 or abs(rel - 0.02) < 1e-5:
                    margin[y, x] = True
                n += 2 * (e <= 2.0) + 2 * (rel <= 0.02)
            conf[y, x] = min(n, 255)
    return conf, margin


def test_confidence_counts(lib):
    sc = cases.scene(80, 60, 4)
    arr = cases.base_problem(sc, 0)
    arr.params.geom_consistency = 1
    ids = [0] + [j for j, _ in sc.pairs[0]][:4]
    rng = np.random.default_rng(3)
    # source depth maps: ground truth, with a rectangle removed (depth 0) and one perturbed by 5 %
    deps = [sc.gt_depth[i].copy() for i in ids]
    deps[1][10:30, 20:50] = 0.0
    deps[2] *= np.float32(1.05)
    arr.depths = deps
    planes = np.zeros((60, 80, 4), np.float32)
    planes[..., 3] = sc.gt_depth[0]
    planes[5:9, 5:15, 3] = -1.0  # ref depth <= 0 -> confidence 0, UNKNOWN
    sel = rng.integers(0, 16, size=(60, 80)).astype(np.uint32)
    weak = np.full((60, 80), A.STRONG, np.uint8)
    conf = np.zeros((60, 80), np.uint8)
    pb = arr.build()
    st = lib.oracle_kat_stage(C.byref(pb), 1, ptr(sel), None, ptr(planes), ptr(weak), ptr(conf), None, None, None)
    assert st == 0
    exp, margin = _confidence_np(arr, planes, sel)
    ok = ~margin
    assert ok.mean() > 0.9
    assert np.array_equal(conf[ok].astype(np.int32), exp[ok])
    assert (conf[5:9, 5:15] == 0).all() and (weak[5:9, 5:15] == A.UNKNOWN).all()
    # the counts cover all outcomes: +1 only (5 % depth error), +5 (consistent), nothing (depth 0)
    assert len(np.unique(conf)) > 8


# ------------------------------------------------------------------------------------------------
# CheckerboardFilterStrong, APD.cu:1711-1855

FILTER_TAPS = [  # (dx, dy, condition on (x, y, W, H)) in the reference's order
    (0, -1, lambda x, y, W, H: y > 0), (0, -3, lambda x, y, W, H: y > 2), (0, -5, lambda x, y, W, H: y > 4),
    (0, 1, lambda x, y, W, H: y < H - 1), (0, 3, lambda x, y, W, H: y < H - 3), (0, 5, lambda x, y, W, H: y < H - 5),
    (-1, 0, lambda x, y, W, H: x > 0), (-3, 0, lambda x, y, W, H: x > 2), (-5, 0, lambda x, y, W, H: x > 4),
    (1, 0, lambda x, y, W, H: x < W - 1), (3, 0, lambda x, y, W, H: x < W - 3), (5, 0, lambda x, y, W, H: x < W - 5),
    (2, -1, lambda x, y, W, H: y > 0 and x < W - 2), (2, 1, lambda x, y, W, H: y < H - 1 and x < W - 2),
    (-2, -1, lambda x, y, W, H: y > 0 and x > 1), (-2, 1, lambda x, y, W, H: y < H - 1 and x > 1),
    (-1, -2, lambda x, y, W, H: x > 0 and y > 2), (1, -2, lambda x, y, W, H: x < W - 1 and y > 2),
    (-1, 2, lambda x, y, W, H: x > 0 and y < H - 2), (1, 2, lambda x, y, W, H: x < W - 1 and y < H - 2),
]


def _filter_np(depth, cost, weak, black_first=True):
    H, W = depth.shape
    d = depth.copy()
    order = (0, 1) if black_first else (1, 0)
    for colour in order:
        new = d.copy()
        for y in range(H):
            for x in range(W):
                if (x + y) % 2 != colour or weak[y, x] == A.WEAK or cost[y, x] < np.float32(0.001):
                    continue
                f = [d[y, x]] + [d[y + dy, x + dx] for dx, dy, ok in FILTER_TAPS
                                 if ok(x, y, W, H) and weak[y + dy, x + dx] == A.STRONG]
                f = np.sort(np.asarray(f, np.float32))
                m = len(f) // 2
                new[y, x] = (f[m - 1] + f[m]) / np.float32(2) if len(f) % 2 == 0 else f[m]
        d = new
    return d


def test_filter_median(lib):
    rng = np.random.default_rng(11)
    W, H = 24, 20
    sc = cases.scene(W, H, 2)
    arr = cases.base_problem(sc, 0)
    depth = rng.integers(1, 200, size=(H, W)).astype(np.float32)
    weak = rng.choice([A.STRONG, A.STRONG, A.STRONG, A.WEAK, A.UNKNOWN], size=(H, W)).astype(np.uint8)
    cost = rng.choice([0.5, 0.5, 0.5, 0.0005], size=(H, W)).astype(np.float32)
    planes = np.zeros((H, W, 4), np.float32)
    planes[..., 3] = depth
    pb = arr.build()
    st = lib.oracle_kat_stage(C.byref(pb), 0, None, ptr(cost), ptr(planes), ptr(weak), None, None, None, None)
    assert st == 0
    exp = _filter_np(depth, cost, weak)
    assert np.array_equal(planes[..., 3], exp)
    assert not np.array_equal(exp, depth)
    # red pixels read the black pixels' filtered depths (all 20 taps are the other colour): the
    # order matters, and the mutated order (red first) disagrees
    assert not np.array_equal(planes[..., 3], _filter_np(depth, cost, weak, black_first=False))


# ------------------------------------------------------------------------------------------------
# FindNearestStrongPoint, APD.cu:2434-2484; GenAnchors + NeigbourUpdate, APD.cu:1857-2100

def _nearest_np(weak, conf):
    H, W = weak.shape
    out = np.full((H, W, 2), -1, np.int32)
    sy, sx = np.nonzero(weak == A.STRONG)
    for y in range(H):
        for x in range(W):
            if weak[y, x] == A.STRONG:
                out[y, x] = (x, y)
                continue
            best = None
            for tx, ty in sorted(zip(sx.tolist(), sy.tolist())):  # the reference's x-major, y-minor order
                if abs(tx - x) > 100 or abs(ty - y) > 100 or conf[ty, tx] < conf[y, x]:
                    continue
                d2 = (tx - x) ** 2 + (ty - y) ** 2
                if best is None or d2 < best[0] or (d2 == best[0] and conf[ty, tx] > best[1]):
                    best = (d2, conf[ty, tx], tx, ty)
            if best is not None:
                out[y, x] = (best[2], best[3])
    return out


def test_find_nearest_strong(lib):
    rng = np.random.default_rng(2)
    W, H = 48, 36
    sc = cases.scene(W, H, 2)
    arr = cases.base_problem(sc, 0)
    weak = rng.choice([A.STRONG, A.WEAK, A.WEAK, A.WEAK, A.WEAK, A.UNKNOWN], size=(H, W)).astype(np.uint8)
    conf = rng.integers(0, 4, size=(H, W)).astype(np.uint8)
    conf[(weak != A.STRONG) & (rng.random((H, W)) < 0.05)] = 9  # above every STRONG point's confidence
    nearest = np.zeros((H, W, 2), np.int16)
    pb = arr.build()
    st = lib.oracle_kat_stage(C.byref(pb), 2, None, None, None, ptr(weak), ptr(conf), ptr(nearest), None, None)
    assert st == 0
    exp = _nearest_np(weak, conf)
    assert np.array_equal(nearest.astype(np.int32), exp)
    # some pixels have no STRONG point of at least their confidence: sparse STRONG map, high confidences
    assert (exp[..., 0] == -1).any()


def _anchor_problem(W, H, rotate_time, strong, depth_of):
    sc = cases.scene(W, H, 2)
    arr = cases.base_problem(sc, 0)
    arr.params.use_APD = 1
    arr.params.state = A.REFINE_ITER
    arr.params.rotate_time = rotate_time
    arr.params.ransac_threshold = 0.01
    arr.depths = list(sc.gt_depth[:len(arr.images)])
    weak = np.full((H, W), A.WEAK, np.uint8)
    planes = np.zeros((H, W, 4), np.float32)
    planes[..., 2] = -1.0
    planes[..., 3] = 5.0
    for (x, y) in strong:
        weak[y, x] = A.STRONG
        planes[y, x, 3] = depth_of((x, y))
    arr.weak_info = weak
    arr.confidence = np.ones((H, W), np.uint8)
    arr.init_planes = planes
    return arr, weak, planes


def _run_anchors(lib, arr, weak, planes):
    W, H = arr.width, arr.height
    wc = int((weak == A.WEAK).sum())
    anchors = np.zeros((wc, 9, 2), np.int16)
    reliable = np.zeros((H, W), np.uint8)
    w = weak.copy()
    conf = arr.confidence.copy()
    pl = planes.copy()  # kept alive across the call
    pb = arr.build()
    st = lib.oracle_kat_stage(C.byref(pb), 3, None, None, ptr(pl), ptr(w), ptr(conf), None, ptr(anchors), ptr(reliable))
    assert st == 0
    return anchors, reliable, w


def _ring(cx, cy, r, dirs=8):
    pts = []
    for k in range(dirs):
        a = 2 * np.pi * k / dirs
        pts.append((int(round(cx + r * np.cos(a))), int(round(cy + r * np.sin(a)))))
    return pts


def test_gen_anchors_coplanar_ring(lib):
    """A WEAK pixel with one STRONG point 20 px away in each of the 8 search directions, all on one
    plane (depth 5): every direction finds its point (the nearest STRONG point of a sample on the
    ray, accepted within the 22.5-degree cone), RANSAC keeps all 8 as inliers (>= 6), so anchors 1..8
    are exactly those points and the pixel stays reliable."""
    cx, cy = 48, 40
    ring = _ring(cx, cy, 20)
    arr, weak, planes = _anchor_problem(96, 80, 1, ring, lambda p: 5.0)
    anchors, reliable, w = _run_anchors(lib, arr, weak, planes)
    k = int(np.nonzero((weak == A.WEAK).ravel())[0].tolist().index(cy * 96 + cx))
    a = anchors[k]
    assert tuple(a[0]) == (cx, cy)
    assert {tuple(p) for p in a[1:].tolist()} == set(ring)
    assert reliable[cy, cx] == 1 and w[cy, cx] == A.WEAK


def test_gen_anchors_off_plane_points_dropped(lib):
    """Same ring, two points off the plane (depth 7): RANSAC's best plane has 6 inliers; the 2
    outliers get weight FLT_MAX and anchors 7, 8 become (-1, -1) (APD.cu:2060-2080)."""
    cx, cy = 48, 40
    ring = _ring(cx, cy, 20)
    off = {ring[1], ring[5]}
    arr, weak, planes = _anchor_problem(96, 80, 1, ring, lambda p: 7.0 if p in off else 5.0)
    anchors, reliable, w = _run_anchors(lib, arr, weak, planes)
    k = int(np.nonzero((weak == A.WEAK).ravel())[0].tolist().index(cy * 96 + cx))
    a = [tuple(p) for p in anchors[k].tolist()]
    assert set(a[1:7]) == set(ring) - off
    assert a[7:] == [(-1, -1), (-1, -1)]
    assert reliable[cy, cx] == 1


def test_gen_anchors_too_few_directions(lib):
    """Only 3 STRONG points (<= 3 directions found, APD.cu:1965-1968): unreliable, and NeigbourUpdate
    turns the pixel UNKNOWN (APD.cu:2084-2100); its anchors stay (self, -1 x 8)."""
    cx, cy = 48, 40
    pts = _ring(cx, cy, 20)[:3]
    arr, weak, planes = _anchor_problem(96, 80, 1, pts, lambda p: 5.0)
    anchors, reliable, w = _run_anchors(lib, arr, weak, planes)
    k = int(np.nonzero((weak == A.WEAK).ravel())[0].tolist().index(cy * 96 + cx))
    assert [tuple(p) for p in anchors[k].tolist()] == [(cx, cy)] + [(-1, -1)] * 8
    assert reliable[cy, cx] == 0 and w[cy, cx] == A.UNKNOWN


def test_gen_anchors_six_coplanar_points(lib):
    """Six coplanar STRONG points in six of the 8 directions: six directions found (> 3), RANSAC's
    plane has exactly 6 inliers (>= 6), so the pixel is reliable with anchors 1..6 = the points and
    anchors 7, 8 = (-1, -1) (sort_small_weighted over 6 entries, APD.cu:2074-2080)."""
    cx, cy = 48, 40
    pts = [p for i, p in enumerate(_ring(cx, cy, 20)) if i not in (2, 6)]
    arr, weak, planes = _anchor_problem(96, 80, 1, pts, lambda p: 5.0)
    anchors, reliable, w = _run_anchors(lib, arr, weak, planes)
    k = int(np.nonzero((weak == A.WEAK).ravel())[0].tolist().index(cy * 96 + cx))
    a = [tuple(p) for p in anchors[k].tolist()]
    assert set(a[1:7]) == set(pts) and a[7:] == [(-1, -1), (-1, -1)]
    assert reliable[cy, cx] == 1 and w[cy, cx] == A.WEAK


def test_gen_anchors_cone(lib):
    """STRONG points at 30, 120, 210 and 300 degrees: the search direction 30 degrees away from a
    point (cos 30 = 0.866) rejects it (threshold cos(22.5) = 0.924, APD.cu:1900, 1939); only the
    direction 15 degrees away accepts it. Four directions found, so RANSAC sees 4 points: fewer
    than 6 inliers, unreliable, UNKNOWN."""
    cx, cy = 48, 40
    pts = [(int(round(cx + 20 * np.cos(np.radians(a)))), int(round(cy + 20 * np.sin(np.radians(a)))))
           for a in (30, 120, 210, 300)]
    arr, weak, planes = _anchor_problem(96, 80, 1, pts, lambda p: 5.0)
    anchors, reliable, w = _run_anchors(lib, arr, weak, planes)
    k = int(np.nonzero((weak == A.WEAK).ravel())[0].tolist().index(cy * 96 + cx))
    assert reliable[cy, cx] == 0 and w[cy, cx] == A.UNKNOWN
    assert [tuple(p) for p in anchors[k].tolist()] == [(cx, cy)] + [(-1, -1)] * 8
