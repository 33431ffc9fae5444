"""GenAnchors search statistics on the bench's headline problem (APD_ANCHOR_STATS build):
APD_LIB=apde-mvs_amd/lib/ab_anchor.so python tools/anchor_stats.py"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import bench
import apd_abi as A
W, H, N = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (6048, 4032, 10)
sc = bench.make_scene(W, H, N, 1, "smooth")
eng = A.Engine(0, A.load_library())
ids = [0] + [j for j, _ in sc.pairs[0]][:N]
priors = bench.first_init_priors(eng, sc, ids, N)
arr = bench.final_round_problem(sc, priors, 0, N)
eng.set_problem(arr)
eng.profile_reset(True)
eng.prepare()
eng.synchronize()
c = (A.C.c_int64 * 64)()
eng._check(eng.lib.apd_profile_counters(eng.ctx, c, 64), "counters")
c = list(c)[32:]  # the instrumented builds' slots (APD_INSTR = 32)
steps = sum(c[20:25])
print(f"lane steps {steps}: success at attempt 1..4 {[c[20 + i] for i in range(4)]}, none {c[24]}; "
      f"wave steps {c[25]} (lane utilisation {steps / max(64 * c[25], 1):.3f}); "
      f"WEAK px {(arr.weak_info == A.WEAK).sum()}, steps per WEAK px {steps / max((arr.weak_info == A.WEAK).sum(), 1):.1f}")
