"""Phase profile of the Weak-path kernels from an instrumented build (-DAPD_PHASE_STAMPS): runs the
bench's headline problem (or AB_W x AB_H, N) once with profiling on and prints each phase's share of
the cycles wave 0 of every workgroup spent (barrier to barrier).
Usage: APD_LIB=apde-mvs_amd/lib/ab_phase.so python tools/phase_profile.py [W H N]"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import bench
import apd_abi as A

W, H, N = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (6048, 4032, 10)
sc = bench.make_scene(W, H, N, 1, os.environ.get("AB_TEXTURE", "smooth"))
eng = A.Engine(0, A.load_library())
ids = [0] + [j for j, _ in sc.pairs[0]][:N]
priors = bench.first_init_priors(eng, sc, ids, N)
arr = bench.final_round_problem(sc, priors, 0, N)
eng.set_problem(arr)
eng.run()  # warm
eng.set_problem(arr)
eng.profile_reset(True)
eng.run()
c = (A.C.c_int64 * 64)()
eng._check(eng.lib.apd_profile_counters(eng.ctx, c, 64), "counters")
c = list(c)[32:]  # the instrumented builds' slots (APD_INSTR = 32)
names = {8: "cand setup (hash, windows)", 9: "cand pair windows", 10: "cand centre windows", 11: "cand focal combination",
         0: "sweep P0 anchors/windows", 1: "sweep P1 current plane", 2: "sweep P2 view selection+geom",
         3: "sweep P3 fit plane", 4: "sweep P4 candidates", 5: "sweep P5 refinement", 6: "sweep P6 acceptance"}
for lo, hi, title in ((8, 12, "k_weak_cand_vm"), (0, 7, "k_sweep_weak_vm")):
    tot = (sum(c[8 + i] for i in range(lo, hi)) + (c[30] if lo == 0 else 0)) or 1
    print(title)
    for i in range(lo, hi):
        print(f"  {names[i]:32s} {100.0 * c[8 + i] / tot:6.1f} %")
    if lo == 0:
        print(f"  {'sweep P2a (before P1b)':32s} {100.0 * c[30] / tot:6.1f} %   (P2 above = P1b + P1c when stamped)")
        print(f"  (of P2a: geometric terms, thread 0's own time {100.0 * c[15] / max(c[30] or c[10], 1):5.1f} %)")
t = eng.timing()
print(f"iteration ms {list(t.iter_ms)[:t.iterations]}")
for slot, what in ((0, "sweep P0 pixels"), (2, "sweep P0 current plane = an anchor candidate's"), (4, "sweep P0 fit plane = current plane"), (6, "sweep P0 fit plane = an anchor candidate's"), (16, "sweep P1c anchor hypothesis taken"), (20, "sweep P5 refinement tasks"), (22, "sweep P3 fit-plane tasks"), (24, "sweep P1b current-plane tasks"),
                   (26, "cand pair-window passes"), (28, "cand centre-window tasks")):
    if c[slot]:
        print(f"{what:32s} waves {c[slot]:>12d}  active lanes {c[slot + 1] / (64.0 * c[slot]):6.3f}")
