"""GenAnchors' filtered direction test (k_gen_anchors, ga_angle_ok): the sum with 1 / sqrt from the
hardware's approximate reciprocal square root decides only outside a 1e-4 band around the threshold,
where it must agree with the IEEE statement (normalize2, then the dot product > thr; APD.cu:1936-1939).
Checked here in IEEE fp32 (numpy) for every direction the search uses (8 rays x rotate_time rotations,
rotate_time 1..4, main.cpp's rounds) and every integer offset up to 256 pixels, with the approximate
reciprocal square root taken 1 ulp below and 1 ulp above the correctly rounded value (v_rsq_f32's
documented error), i.e. the filter's verdict equals the IEEE verdict wherever it is used. CPU only."""
import numpy as np

f32 = np.float32


def normalize2(x, y):
    ns = f32(x * x) + f32(y * y)
    inv = f32(1.0) / np.sqrt(ns, dtype=np.float32)
    return f32(x * inv), f32(y * inv)


def directions(rotate_time):
    """The search's ray directions in the kernel's fp32 statements (k_gen_anchors, APD.cu:1903-1958)."""
    angle = f32(45.0) / f32(rotate_time)
    c = f32(np.cos(np.float64(angle) * np.pi / 180.0))
    s = f32(np.sin(np.float64(angle) * np.pi / 180.0))
    thr = f32(np.cos(np.float64(angle / f32(2.0)) * np.pi / 180.0))
    out = []
    for odx in (-1, 0, 1):
        for ody in (-1, 0, 1):
            if odx == 0 and ody == 0:
                continue
            dx, dy = normalize2(f32(odx), f32(ody))
            for _ in range(rotate_time):
                out.append((dx, dy))
                rx = f32(f32(dx * c) - f32(dy * s))
                ry = f32(f32(dx * s) + f32(dy * c))
                dx, dy = normalize2(rx, ry)
    return out, thr


def test_filtered_direction_test_agrees_with_ieee():
    R = 256
    t = np.arange(-R, R + 1, dtype=np.float32)
    tx, ty = np.meshgrid(t, t, indexing="ij")
    keep = (tx != 0) | (ty != 0)
    tx, ty = tx[keep], ty[keep]
    ns = (tx * tx).astype(np.float32) + (ty * ty).astype(np.float32)
    inv = (f32(1.0) / np.sqrt(ns, dtype=np.float32)).astype(np.float32)
    exact_rsq = (1.0 / np.sqrt(ns.astype(np.float64))).astype(np.float32)  # correctly rounded 1 / sqrt
    nx, ny = (tx * inv).astype(np.float32), (ty * inv).astype(np.float32)
    decided = 0
    for rt in (1, 2, 3, 4):
        dirs, thr = directions(rt)
        for dx, dy in dirs:
            ieee = ((nx * dx).astype(np.float32) + (ny * dy).astype(np.float32)) > thr
            for r in (np.nextafter(exact_rsq, np.float32(0)), exact_rsq, np.nextafter(exact_rsq, np.float32(np.inf))):
                va = ((tx * r).astype(np.float32) * dx).astype(np.float32) + ((ty * r).astype(np.float32) * dy).astype(np.float32)
                outside = np.abs(va - thr) > f32(1e-4)
                assert np.array_equal(ieee[outside], (va > thr)[outside])
                decided += int(outside.sum())
    assert decided > 0.99 * 3 * sum(len(directions(rt)[0]) for rt in (1, 2, 3, 4)) * tx.size
