"""bench.py's roofline.traffic source: the newest PMC summary under profiles/ for the measured kernel
and shape, never an unrelated counter study that merely sorts last (CPU only)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def _write(d, name, obj):
    with open(os.path.join(d, name), "w") as f:
        json.dump(obj, f)


def test_latest_pmc_skips_other_studies(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    good = {"kernel": "k_sweep_strong", "width": 3024, "n_src": 8, "hbm_bytes_per_launch": 1.0}
    newer = dict(good, hbm_bytes_per_launch=2.0)
    _write(prof, "r2_pmc_sweep_strong.json", good)
    _write(prof, "r2_s7_pmc_sweep_strong.json", newer)
    # sorts last but is a per-shape TCP study without the kernel/shape keys
    _write(prof, "r2_zz_pmc_tcp_study.json", {"3024x2016": {"n_src": 8}})
    # right kernel, other shape
    _write(prof, "r3_pmc_sweep_strong_c3.json", dict(good, width=6048, hbm_bytes_per_launch=9.0))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.latest_pmc("k_sweep_strong", 3024, 8)["hbm_bytes_per_launch"] == 2.0
    assert bench.latest_pmc("k_sweep_strong", 6048, 8)["hbm_bytes_per_launch"] == 9.0
    assert bench.latest_pmc("k_sweep_strong", 3024, 10) is None


def test_committed_profiles_give_traffic():
    pmc = bench.latest_pmc("k_sweep_strong", 3024, 8)
    assert pmc is not None and pmc["hbm_bytes_per_launch"] > 0
