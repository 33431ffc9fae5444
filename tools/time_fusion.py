"""Time the fusion of the `apd` binary (HIP kernels + host ordered commit) on a synthetic scan at
the benchmark resolution, and the C oracle (the reference's loops restated, single-threaded apart
from WeakVisFilter's per-view threads) on the same scan; checks that both write the same APD.ply.

    python tools/time_fusion.py --width 3024 --height 2016 --views 9 --dataset ETH3D [--oracle]

Prints one JSON line. The scan (~1 GB at the default size) goes to a temporary directory.
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "apde-mvs_amd")]

import fusion_lib as FL  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3024)
    ap.add_argument("--height", type=int, default=2016)
    ap.add_argument("--views", type=int, default=9)
    ap.add_argument("--dataset", default="ETH3D")
    ap.add_argument("--weak_filter", type=int, default=1)
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--scan_only", default="", help="only write the scan into this folder (for rocprofv3 runs)")
    a = ap.parse_args()
    tmp = a.scan_only or tempfile.mkdtemp(prefix="fscan_")
    t0 = time.time()
    FL.make_fusion_scan(tmp, a.width, a.height, a.views - 1, seed=3)
    gen_s = time.time() - t0
    if a.scan_only:
        print(json.dumps({"scan": tmp, "scan_gen_s": round(gen_s, 2)}))
        return
    res = dict(workload=f"fusion {a.dataset}, {a.views} views at {a.width}x{a.height}, weak_filter={a.weak_filter}",
               scan_gen_s=round(gen_s, 2))
    walls = []
    for _ in range(a.repeat):
        t0 = time.time()
        r = subprocess.run([FL.APD_BIN, "--dense_folder", tmp, "--dataset", a.dataset, "--only_fuse", "true",
                            "--weak_filter", "true" if a.weak_filter else "false"],
                           capture_output=True, text=True, timeout=900)
        walls.append(time.time() - t0)
        if r.returncode != 0:
            print(r.stdout[-2000:], r.stderr[-2000:], file=sys.stderr)
            sys.exit(1)
    m = re.search(r"Fusion: (\d+) points, load (\d+) ms, upload (\d+) ms, weak filter (\d+) ms, fuse (\d+) ms "
                  r"\(device (\d+) ms, terms (\d+) ms, commit (\d+) ms\), write (\d+) ms", r.stdout)
    keys = ["points", "load_ms", "upload_ms", "filter_ms", "fuse_ms", "device_ms", "terms_ms", "commit_ms", "write_ms"]
    res.update({k: int(v) for k, v in zip(keys, m.groups())})
    res["apd_wall_s"] = round(min(walls), 3)
    px = a.width * a.height * a.views
    res["mpix_s_fuse"] = round(px / ((res["filter_ms"] + res["fuse_ms"]) / 1e3) / 1e6, 2)
    if a.oracle:
        hl = FL.hostlib()
        views = FL.load_views(tmp, hl)
        t0 = time.time()
        xyz, col, _, _ = FL.run_oracle(views, a.dataset, bool(a.weak_filter))
        res["oracle_s"] = round(time.time() - t0, 2)
        res["oracle_points"] = int(len(xyz))
        got = open(os.path.join(tmp, "APD", "APD.ply"), "rb").read()
        res["ply_identical"] = got == FL.ply_bytes(xyz, col)
        res["mpix_s_oracle"] = round(px / res["oracle_s"] / 1e6, 3)
    print(json.dumps(res))
    subprocess.run(["rm", "-rf", tmp])


if __name__ == "__main__":
    main()
