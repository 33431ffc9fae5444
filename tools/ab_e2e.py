"""A/B of whole RunPatchMatch runs between library builds, interleaved in one process (HIP-event
breakdown from apd_get_timing). Usage: python tools/ab_e2e.py libA.so libB.so [...]"""
import os, sys, statistics
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import apd_abi as A, synth

W, H, N = int(os.environ.get("AB_W", 3024)), int(os.environ.get("AB_H", 2016)), int(os.environ.get("AB_N", 8))
ROUNDS = int(os.environ.get("AB_ROUNDS", 3))
sc = synth.make_scene(W, H, N)
arr = A.scene_problem(sc, 0, [j for j, _ in sc.pairs[0]][:N])
engines = []
for path in sys.argv[1:]:
    e = A.Engine(0, A.load_library(path))
    e.set_problem(arr)
    e.run()
    engines.append((os.path.basename(path), e))
res = {n: [] for n, _ in engines}
for r in range(ROUNDS):
    for name, e in engines:
        e.set_problem(arr)
        e.run()
        t = e.timing()
        res[name].append((t.total_ms, t.prepare_ms, t.sweep_ms, t.post_ms))  # (total = prepare + sweep + post)
for name, v in res.items():
    med = [statistics.median(x[i] for x in v) for i in range(4)]
    print(f"{name}: total {med[0]:.2f} ms  prepare {med[1]:.2f}  sweep {med[2]:.2f}  post {med[3]:.2f}", flush=True)
