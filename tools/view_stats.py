"""Selected-view and view-weight statistics of one RunPatchMatch on the bench scene."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import apd_abi as A, synth
W, H, N = int(os.environ.get("AB_W", 3024)), int(os.environ.get("AB_H", 2016)), int(os.environ.get("AB_N", 8))
sc = synth.make_scene(W, H, N)
arr = A.scene_problem(sc, 0, [j for j, _ in sc.pairs[0]][:N])
e = A.Engine(0)
e.set_problem(arr); e.run()
o = e.results(A.Outputs(W, H, N))
sel = o.selected_views
pc = np.zeros(sel.shape, np.int32)
for k in range(N):
    pc += ((sel >> k) & 1).astype(np.int32)
vw = o.view_weights
print(f"selected views per pixel: mean {pc.mean():.2f} of {N}; hist {np.bincount(pc.ravel(), minlength=N+1).tolist()}")
print(f"views with weight > 0 per pixel: mean {(vw > 0).sum(0).mean():.2f}")
print(f"weak state: {np.bincount(o.weak_info.ravel(), minlength=3).tolist()}")
