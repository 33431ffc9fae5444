"""Diagnostic: per-case bit-level diff report HIP vs oracle, plus a timing probe. Run on the GPU box."""
import os, sys, time
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "apde-mvs_amd")]
import numpy as np
import apd_abi as A, cases, oracle_lib, synth

lib = oracle_lib.load()
orun = lambda arr: oracle_lib.run(lib, arr)
names = sys.argv[1:] or list(cases.CASES)
eng = A.Engine(0) if A.load_library().apd_device_count() > 0 else None
for name in names:
    arr = cases.make_case(name, orun)
    t = time.time(); ref = orun(arr); to = time.time() - t
    if eng is None:
        print(name, "oracle only", f"{to:.2f}s", flush=True); continue
    eng.set_problem(arr); eng.run()
    got = eng.results(A.Outputs(arr.width, arr.height, len(arr.images) - 1, max_weak=arr.width * arr.height))
    d = cases.compare(ref, got)
    print(name, d, f"oracle {to:.2f}s hip {eng.timing().total_ms:.2f}ms", flush=True)
    for f, n in d.items():
        if n:
            x, y = getattr(ref, f), getattr(got, f)
            if x.dtype.kind == 'f':
                bad = ~((x.view(np.uint32) == y.view(np.uint32)) | (np.isnan(x) & np.isnan(y)))
            else:
                bad = x != y
            idx = np.argwhere(bad)[:3]
            print("   ", f, [(tuple(int(v) for v in i), x[tuple(i)], y[tuple(i)]) for i in idx], flush=True)
