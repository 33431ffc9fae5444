"""A/B timing of the Strong sweep between library builds, interleaved in ONE process on one device
(cdna_hip_programming.md §5.4 rule 24). Usage: python tools/ab_sweep.py libA.so libB.so [...]
Prints per build the median/min per-iteration ms (HIP events) over R interleaved rounds."""
import os, sys, time, statistics
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import apd_abi as A, synth

W, H, N = int(os.environ.get("AB_W", 3024)), int(os.environ.get("AB_H", 2016)), int(os.environ.get("AB_N", 8))
ROUNDS = int(os.environ.get("AB_ROUNDS", 5))
sc = synth.make_scene(W, H, N)
arr = A.scene_problem(sc, 0, [j for j, _ in sc.pairs[0]][:N])
engines = []
for spec in sys.argv[1:]:
    path, _, opt = spec.partition(":")   # "lib.so:f32" = fp32 quad texels; "lib.so:ENV=VAL,..." = env at create
    envs = {}
    if opt == "f32":
        envs["APD_TEX_F32"] = "1"
    elif opt:
        envs = dict(kv.split("=", 1) for kv in opt.split(","))
    for k, v in envs.items():
        os.environ[k] = v
    lib = A.load_library(path)
    e = A.Engine(0, lib)
    e.set_problem(arr)
    for k in envs:
        os.environ.pop(k, None)
    e.prepare()
    e.iteration(0)
    e.synchronize()
    engines.append((os.path.basename(path) + (':' + opt if opt else ''), e))
res = {n: [] for n, _ in engines}
for r in range(ROUNDS):
    for name, e in engines:
        e.profile_reset(True)
        for i in range(3):
            e.iteration(i)
        ms, launches, _ = e.profile_query()
        res[name].append(ms / launches)
for name, v in res.items():
    print(f"{name}: sweep launch median {statistics.median(v):.3f} ms  min {min(v):.3f} ms  "
          f"per-iter {2*statistics.median(v):.2f} ms  ({W*H/(2*statistics.median(v)*1e-3)/1e6:.1f} Mpix/s)", flush=True)
