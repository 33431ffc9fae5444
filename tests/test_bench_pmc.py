"""bench.py's roofline.traffic source: the newest PMC summary under profiles/ for the measured kernel
and shape collected from the current kernel sources (source hash), never an unrelated counter study
or another build's summary that merely sorts last (CPU only)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def _write(d, name, obj):
    with open(os.path.join(d, name), "w") as f:
        json.dump(obj, f)


def _tree(tmp_path):
    """a stand-in repo with kernel sources of its own (their hash keys the summaries)"""
    for f in bench.KERNEL_SOURCES:
        p = tmp_path / f
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text("// " + f)
    prof = tmp_path / "profiles"
    prof.mkdir()
    return prof


def test_latest_pmc_skips_other_studies(tmp_path, monkeypatch):
    prof = _tree(tmp_path)
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    h = bench.source_hash()
    good = {"kernel": "k_sweep_strong", "width": 3024, "n_src": 8, "hbm_bytes_per_launch": 1.0, "source_hash": h}
    newer = dict(good, hbm_bytes_per_launch=2.0)
    _write(prof, "r2_pmc_sweep_strong.json", good)
    _write(prof, "r2_s7_pmc_sweep_strong.json", newer)
    # sorts last but is a per-shape TCP study without the kernel/shape keys
    _write(prof, "r2_zz_pmc_tcp_study.json", {"3024x2016": {"n_src": 8}})
    # right kernel, other shape
    _write(prof, "r3_pmc_sweep_strong_c3.json", dict(good, width=6048, hbm_bytes_per_launch=9.0))
    assert bench.latest_pmc("k_sweep_strong", 3024, 8)["hbm_bytes_per_launch"] == 2.0
    assert bench.latest_pmc("k_sweep_strong", 6048, 8)["hbm_bytes_per_launch"] == 9.0
    assert bench.latest_pmc("k_sweep_strong", 3024, 10) is None


def test_latest_pmc_refuses_other_builds(tmp_path, monkeypatch):
    """A summary collected from other kernel sources (an older round, a superseded variant that sorts
    last by name) or without a hash is never the current traffic: None, and bench reports null."""
    prof = _tree(tmp_path)
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    h = bench.source_hash()
    base = {"kernel": "k_sweep_weak_vm", "width": 6048, "n_src": 10, "hbm_bytes_per_launch": 1.0}
    _write(prof, "r5_pmc_k_sweep_weak_vm_c3.json", dict(base, source_hash=h))
    _write(prof, "r5_pmc_k_sweep_weak_vm_c3_occ3.json", dict(base, hbm_bytes_per_launch=7.0, source_hash="0" * 16))
    _write(prof, "r6_pmc_k_sweep_weak_vm_c3_nohash.json", dict(base, hbm_bytes_per_launch=8.0))
    assert bench.latest_pmc("k_sweep_weak_vm", 6048, 10)["hbm_bytes_per_launch"] == 1.0
    (tmp_path / bench.KERNEL_SOURCES[0]).write_text("// edited after the collection")
    assert bench.source_hash() != h
    assert bench.latest_pmc("k_sweep_weak_vm", 6048, 10) is None


def test_committed_pmc_summaries_are_keyed():
    """Every committed summary bench could report either carries a 16-hex source hash or predates the
    keying (round <= 5) and therefore can never match."""
    import glob
    import re
    for f in glob.glob(os.path.join(REPO, "profiles", "*pmc*.json")):
        d = json.load(open(f))
        if not isinstance(d, dict) or "hbm_bytes_per_launch" not in d:
            continue
        h = d.get("source_hash")
        assert h is None or re.fullmatch(r"[0-9a-f]{16}", h), f
        if h is None:
            assert re.match(r"r[1-5]_", os.path.basename(f)), f
