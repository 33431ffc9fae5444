import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "apde-mvs_amd")]
import numpy as np
import apd_abi as A, cases, oracle_lib
lib = oracle_lib.load(); orun = lambda arr: oracle_lib.run(lib, arr)
arr = cases.make_case(sys.argv[1] if len(sys.argv) > 1 else "refine_init_apd", orun)
for iters in [0, 1, 2, 3]:
    arr.params.max_iterations = iters
    ref = orun(arr)
    eng = A.Engine(0); eng.set_problem(arr); eng.run()
    got = eng.results(A.Outputs(arr.width, arr.height, len(arr.images) - 1, max_weak=arr.width * arr.height))
    eng.close()
    d = cases.compare(ref, got)
    wc = int(ref.weak_count[0])
    anc_eq = np.array_equal(ref.anchors[:wc], got.anchors[:wc])
    print("iters", iters, d, "anchors equal", anc_eq, flush=True)
    if not anc_eq:
        bad = np.argwhere((ref.anchors[:wc] != got.anchors[:wc]).any(-1).any(-1))[:5].ravel()
        for b in bad:
            print("  anchor row", b, ref.anchors[b].tolist(), got.anchors[b].tolist())
    x = ref.planes.view(np.uint32); y = got.planes.view(np.uint32)
    bad = np.argwhere((x != y).any(-1))
    inw = arr.weak_info
    for (yy, xx) in bad[:6]:
        print("  px", (int(xx), int(yy)), "in_weak", inw[yy, xx], "ref", ref.planes[yy, xx], "got", got.planes[yy, xx], "cost", ref.costs[yy, xx], got.costs[yy, xx])
