"""A/B of one APD pass (REFINE_ITER + use_APD + geometric consistency, main.cpp round >= 1) between
library builds, interleaved in one process. Priors come from FIRST_INIT runs of the neighbouring
views (first library), as in tools/time_apd_pass.py. Prints the HIP-event breakdown per build and
whether every build's outputs are bit-identical to the first's.
Usage: python tools/ab_apd.py libA.so[:ENV=VAL,...] libB.so [...]   (AB_W / AB_H / AB_N / AB_ROUNDS / AB_SA;
AB_FIRST=1 times a FIRST_INIT problem instead; AB_TEXTURE=rich the texture-rich scene)"""
import os, sys, statistics
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import apd_abi as A, synth, cases

W, H, N = int(os.environ.get("AB_W", 3024)), int(os.environ.get("AB_H", 2016)), int(os.environ.get("AB_N", 8))
ROUNDS = int(os.environ.get("AB_ROUNDS", 3))
sc = synth.make_scene(W, H, N, texture=os.environ.get("AB_TEXTURE", "smooth"))  # AB_TEXTURE=rich: the texture-rich variant


def make_engine(spec):
    path, _, opt = spec.partition(":")
    envs = dict(kv.split("=", 1) for kv in opt.split(",")) if opt else {}
    os.environ.update(envs)
    e = A.Engine(0, A.load_library(path))
    for k in envs:
        os.environ.pop(k, None)
    return os.path.basename(path) + (":" + opt if opt else ""), e


engines = [make_engine(s) for s in sys.argv[1:]]
e0 = engines[0][1]


def run(e, arr):
    e.set_problem(arr)
    e.run()
    return e.results(A.Outputs(arr.width, arr.height, len(arr.images) - 1))


if os.environ.get("AB_FIRST") == "1":
    arr = cases.base_problem(sc, 0, N)
else:
    priors = [run(e0, cases.base_problem(sc, r, N)) for r in range(len(sc.images))]
    arr = cases.refine_problem(sc, priors, 0, N, state=A.REFINE_ITER, geom=True, apd=True,
                               sa=os.environ.get("AB_SA") == "1")  # AB_SA=1: the scene's plane labels as SA masks
    if os.environ.get("AB_FINAL") == "1":  # bench.py's headline pass: main.cpp's last round (rotate_time 4)
        arr.params.rotate_time, arr.params.ransac_threshold, arr.params.weak_peak_radius = 4, 0.01 - 3 * 0.00125, 4
outs = {}
res = {n: [] for n, _ in engines}
for r in range(ROUNDS):
    for name, e in engines:
        out = run(e, arr)
        t = e.timing()
        # (prepare_ms: the prepare bracket; RandomInitialization runs beside the lists and the pair
        # table on a side stream, so init_ms is not a serial phase of the total)
        res[name].append((t.total_ms, t.anchors_ms, t.prepare_ms, t.sweep_ms, t.post_ms,
                          statistics.median(list(t.iter_ms)[:t.iterations])))
        outs.setdefault(name, out)
ref = outs[engines[0][0]]
for name, v in res.items():
    med = [statistics.median(x[i] for x in v) for i in range(6)]
    d = cases.compare(ref, outs[name])
    print(f"{name}: total {med[0]:.1f} ms  anchors {med[1]:.1f}  prepare {med[2]:.1f}  sweep {med[3]:.1f}  "
          f"post {med[4]:.1f}  iter {med[5]:.2f} ({W * H / med[5] / 1e3:.2f} Mpix/s)  identical={not any(d.values())}",
          flush=True)
