"""Diagnose fusion kernel vs oracle differences on the test scan (GPU box)."""
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "apde-mvs_amd")]
import apd_abi as A  # noqa: E402
import fusion_lib as FL  # noqa: E402

d = tempfile.mkdtemp()
FL.make_fusion_scan(d, 96, 72, 4, seed=11)
hl = FL.hostlib()
views = FL.load_views(d, hl)
eng = A.FusionEngine(0)
eng.set_views(views)
q_view = hl.apdhost_view_cut_deg(80.0)
q_angle = hl.apdhost_angle_cut_lt(np.float32(0.174533))
print("q_view", repr(q_view), "q_angle", repr(q_angle))
for i in range(len(views)):
    got = eng.weak_filter(i, q_view)
    exp = FL.oracle_weak_filter(views, i)
    diff = np.argwhere(got != exp)
    print(f"view {i}: weak filter diffs {len(diff)} (gpu set {int(got.sum())}, oracle set {int(exp.sum())})")
    for r, c in diff[:4]:
        conf = views[i]["conf"]
        W = conf.shape[1]
        flat = conf.ravel()
        o = r * W + 4 * c
        b = [int(flat[o + k]) if o + k < flat.size else 0 for k in range(4)]
        f = np.array(b, np.uint8).view(np.float32)[0]
        print(f"   px ({r},{c}) gpu {got[r, c]} oracle {exp[r, c]} ref conf bytes {b} -> {f!r} weak {views[i]['weak'][r, c]}"
              f" depth {views[i]['depth'][r, c]!r}")
    src = [j for j in range(len(views)) if j != i]
    sp, dist, rel, ang, q = FL.oracle_candidates(views, i, src)
    pix, er, qq = eng.consistency(i, src, q_angle)
    live = (views[i]["depth"] > 0)[..., None] & np.ones(len(src), bool)
    valid = (sp >= 0) & live
    cons = valid & (dist < 2.0) & (rel < np.float32(0.01)) & (ang < np.float32(0.174533))
    exp_pix = np.where(cons, sp, -1)
    bad = (pix != exp_pix) & live
    print(f"   consistency pix diffs {int(bad.sum())} of {int(live.sum())}; valid {int(valid.sum())} cons {int(cons.sum())}")
    erx = dist + np.float32(200) * rel
    bq = valid & (qq.view(np.uint32) != q.view(np.uint32))
    be = valid & (er.view(np.uint32) != erx.view(np.uint32))
    print(f"   q bit diffs {int(bq.sum())}, err_rel bit diffs {int(be.sum())}")
    for idx in np.argwhere(bq)[:3]:
        t = tuple(idx)
        print(f"     q gpu {qq[t]!r} oracle {q[t]!r}")
    for idx in np.argwhere(be)[:3]:
        t = tuple(idx)
        print(f"     er gpu {er[t]!r} oracle {erx[t]!r} dist {dist[t]!r} rel {rel[t]!r}")
    for idx in np.argwhere(bad)[:3]:
        t = tuple(idx)
        print(f"     pix gpu {pix[t]} oracle-sp {sp[t]} cons {cons[t]} dist {dist[t]!r} rel {rel[t]!r} ang {ang[t]!r} q {q[t]!r}")
