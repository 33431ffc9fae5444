"""How many Weak-refinement evaluations (fit plane + 5 candidates per refining WEAK pixel) exact lower
bounds could reject before their anchor windows: runs the bench's headline pass (final-round
REFINE_ITER + APD + geom) on a small rendering of the same scene through the oracle's measurement
build (oracle/liboracle_ws.so, ORACLE_WEAK_STATS). CPU only.
Usage: python tools/weak_bound_stats.py [W H N]"""
import os, sys
from types import SimpleNamespace
import ctypes as C
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import bench
import apd_abi as A

W, H, N = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (378, 252, 10)
os.environ["APD_ORACLE_SO"] = os.path.join(REPO, "oracle", "liboracle_ws.so")
import oracle_lib
lib = oracle_lib.load()
lib.oracle_weak_stats.restype = C.c_longlong
lib.oracle_weak_stats.argtypes = [C.c_int]
sc = bench.make_scene(W, H, N, 1, os.environ.get("AB_TEXTURE", "smooth"))
ids = [0] + [j for j, _ in sc.pairs[0]][:N]
priors = {}
for r in ids:
    out = oracle_lib.run(lib, A.scene_problem(sc, r, [j for j, _ in sc.pairs[r]][:N], seed=0x5EED ^ r))
    priors[r] = SimpleNamespace(planes=out.planes, weak_info=out.weak_info, confidence=out.confidence)
arr = bench.final_round_problem(sc, priors, 0, N)
lib.oracle_weak_stats_reset()
oracle_lib.run(lib, arr)
s = [lib.oracle_weak_stats(i) for i in range(8)]
print(f"{W}x{H} N={N}: candidates {s[0]} (accepted-or-not-exited {s[6]}), weighted-view evaluations {s[1]}, "
      f"with the per-view prefix exit {s[2]} ({s[2] / max(s[1], 1):.3f})")
print(f"  rejected by the geometric bound: {s[3]} ({s[3] / max(s[0], 1):.3f}); by centre + geometric: {s[4]} "
      f"({s[4] / max(s[0], 1):.3f})")
print(f"  anchor-window evaluations: prefix exit {s[2]}, centre+geom bound then prefix exit {s[5]} "
      f"({s[5] / max(s[2], 1):.3f} of the prefix exit's); centre windows for the bound {s[1]}")
