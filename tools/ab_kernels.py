"""Per-kernel HIP-event times of the bench's headline pass (or AB_W x AB_H, AB_N) for several library
builds, one process: python tools/ab_kernels.py libA.so libB.so[:ENV=VAL,...] ..."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import bench
import apd_abi as A

W, H, N = int(os.environ.get("AB_W", 6048)), int(os.environ.get("AB_H", 4032)), int(os.environ.get("AB_N", 10))
sc = bench.make_scene(W, H, N, 1, os.environ.get("AB_TEXTURE", "smooth"))
def make_engine(spec):  # lib.so[:ENV=VAL,...] (env read by apd_create)
    path, _, opt = spec.partition(":")
    envs = dict(kv.split("=", 1) for kv in opt.split(",")) if opt else {}
    os.environ.update(envs)
    e = A.Engine(0, A.load_library(path))
    for k in envs:
        os.environ.pop(k, None)
    return os.path.basename(path) + (":" + opt if opt else ""), e


engs = [make_engine(p) for p in sys.argv[1:]]
ids = [0] + [j for j, _ in sc.pairs[0]][:N]
priors = bench.first_init_priors(engs[0][1], sc, ids, N)
arr = bench.final_round_problem(sc, priors, 0, N)
kinds = {"strong": A.PROF_STRONG_SWEEP, "ransac": A.PROF_RANSAC_FIT, "cand": A.PROF_WEAK_CAND, "weak": A.PROF_WEAK_SWEEP,
         "gp_cost": A.PROF_GP_COST, "cand_g": A.PROF_WEAK_CAND_G, "comb": A.PROF_WEAK_CAND_COMB,
         "dtw": A.PROF_DEPTH_TO_WEAK}
for rnd in range(2):
    for name, e in engs:
        e.set_problem(arr)
        e.run()
        e.set_problem(arr)
        e.profile_reset(True)
        e.run()
        t = e.timing()
        ks = {k: e.profile_kernel(v) for k, v in kinds.items()}
        e.profile_reset(False)
        print(f"{name}: iter {sorted(list(t.iter_ms)[:t.iterations])[t.iterations // 2]:.2f} ms  " +
              "  ".join(f"{k} {ms / max(n, 1):.2f}" for k, (ms, n, _) in ks.items()), flush=True)
