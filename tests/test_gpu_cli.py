"""GPU: the `apd` binary (apde-mvs_amd/host) over a synthetic MVSNet scan, whole reference schedule.

The scan is 1000x750 with 5 views, so main.cpp's schedule has 2 rounds: FIRST_INIT + 3 geometric
passes at 500x375, then REFINE_INIT with APD (anchors, RANSAC, weak sweep, SA masks) + 3 geometric
APD passes at full size. Every view's final depths.bin / normals.bin / weak.bin / confidence.bin must
equal, bit for bit, the same schedule restated in Python (tests/host_schedule.py) driving the HIP
library directly -- which the parity tests tie to the oracle. This checks the whole host side:
image decode + resize, cam parsing, K scaling, prior resizing, anchors map, epilogue, bin-mat
files, seeds, the sequential vs jacobi pass orderings (jacobi on two device contexts), and the
single-context device-resident state (images and priors kept in HBM) against the host-upload path.
"""
import os
import subprocess

import numpy as np
import pytest

import apd_abi as A
import host_schedule as HS
import synth

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APD_BIN = os.path.join(REPO, "apde-mvs_amd", "host", "build", "apd")


@pytest.fixture(scope="module")
def engine():
    lib = A.load_library()
    if lib.apd_device_count() < 1:
        pytest.fail("no HIP device visible")
    eng = A.Engine(0, lib)
    yield eng
    eng.close()


@pytest.fixture(scope="module")
def scan(tmp_path_factory):
    sc = synth.make_scene(1000, 750, 4, seed=7)
    folder = str(tmp_path_factory.mktemp("scan"))
    HS.write_dense_folder(sc, folder, ext=".png", masks=True)
    return folder


def run_engine(engine):
    def fn(arr):
        engine.set_problem(arr)
        engine.run()
        return engine.results(A.Outputs(arr.width, arr.height, len(arr.images) - 1))
    return fn


def check_outputs(folder, expected):
    for ref, exp in expected.items():
        d = os.path.join(folder, "APD", f"{ref:08d}")
        depth = synth.read_bin_mat(os.path.join(d, "depths.bin"))
        normal = synth.read_bin_mat(os.path.join(d, "normals.bin"))
        weak = synth.read_bin_mat(os.path.join(d, "weak.bin"))
        conf = synth.read_bin_mat(os.path.join(d, "confidence.bin"))
        assert np.array_equal(depth.view(np.uint32), exp["depth"].view(np.uint32)), f"depth of view {ref}"
        assert np.array_equal(normal.view(np.uint32), exp["normal"].view(np.uint32)), f"normal of view {ref}"
        assert np.array_equal(weak, exp["weak"]), f"weak of view {ref}"
        assert np.array_equal(conf, exp["conf"]), f"confidence of view {ref}"
        assert (depth > 0).mean() > 0.5


@pytest.mark.parametrize("ordering,gpus,device_state", [
    ("sequential", "0", "1"),   # one context: images and depth/plane priors resident in HBM
    ("sequential", "0", "0"),   # APD_DEVICE_STATE=0: every input uploaded from the host per problem
    ("jacobi", "0", "1"),       # resident state with this pass's maps held back until the pass ends
    ("jacobi", "0,0", "1"),     # two contexts, a device store each; the pass's new maps exchanged at the commit
    ("jacobi", "0,0", "0"),     # two contexts, host-side state
    ("jacobi", "0,0", "oomlib"),  # a library buffer fails after RandomInitialization started on a side stream:
                                  # that context's store is released, the other keeps its own; same outputs
    ("sequential", "0", "cap"),  # device store capped (APD_DEVICE_STATE_CAP_MB): views that do not fit
    ("jacobi", "0", "cap"),      # ... fall back to the host store, same outputs
    ("sequential", "0", "oom"),  # a problem finds HBM exhausted (APD_TEST_ENOMEM_AT): the store is released
    ("jacobi", "0", "oom"),      # and the run continues from the host store, same outputs
])
def test_cli_matches_schedule(scan, engine, ordering, gpus, device_state, tmp_path):
    import shutil
    folder = str(tmp_path / "run")
    shutil.copytree(scan, folder)
    env = dict(os.environ, APD_DEVICE_STATE="1" if device_state in ("cap", "oom", "oomlib") else device_state)
    if device_state == "cap":  # room for the round's images and a few views' maps, not for all of them
        env["APD_DEVICE_STATE_CAP_MB"] = "40"
    if device_state == "oom":  # the 13th problem (second round, maps and images resident) runs out
        env["APD_TEST_ENOMEM_AT"] = "13"
    if device_state == "oomlib":  # the second APD problem (round 1) fails inside apd_stage_prepare
        env["APD_TEST_LIB_ENOMEM_AT"] = "2"
    r = subprocess.run([APD_BIN, "--dense_folder", folder, "--dataset", "ETH3D", "--no_fuse", "true",
                        "--memory_cache", "false", "--gpus", gpus, "--ordering", ordering],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "Round nums: 2" in r.stdout
    resident = device_state in ("1", "cap", "oomlib")
    if device_state == "cap":
        assert "falls back to the host store" in r.stdout
    if device_state in ("oom", "oomlib"):
        assert "device-resident state released" in r.stdout
    assert ("Device-resident state:" in r.stdout) == resident
    assert r.stdout.count("RunPatchMatch time:") == 5 * 8
    expected = HS.run_schedule(folder, run_engine(engine), ordering=ordering)
    check_outputs(folder, expected)


def test_cli_memory_cache_flush(scan, tmp_path):
    """--memory_cache true: nothing reaches the disk until the final flush (--no_fuse forces it)."""
    import shutil
    folder = str(tmp_path / "run")
    shutil.copytree(scan, folder)
    r = subprocess.run([APD_BIN, "--dense_folder", folder, "--no_fuse", "true", "--memory_cache", "true",
                        "--export_anchor", "true", "--export_curve", "true"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "Write memory cache to disk!" in r.stdout
    d = os.path.join(folder, "APD", "00000000")
    for f in ("depths.bin", "normals.bin", "weak.bin", "confidence.bin", "anchors.bin", "anchors_map.bin",
              "reliable_curve.bin"):
        assert os.path.exists(os.path.join(d, f)), f
    hdr = np.fromfile(os.path.join(d, "reliable_curve.bin"), np.int32, 3)
    assert list(hdr) == [1000, 750, 61]
    am = synth.read_bin_mat(os.path.join(d, "anchors_map.bin"))
    n_weak, k = np.fromfile(os.path.join(d, "anchors.bin"), np.int32, 2)
    assert k == 9 and n_weak == int((am >= 0).sum())


def test_run_scans_drives_the_binary(tmp_path):
    """run_scans.py (run.py's orchestration) runs the apd binary over a batch: every scan ends with
    its depth maps and APD/APD.ply, and the log run.py would keep."""
    import sys
    root = tmp_path / "ETH3D"
    root.mkdir()
    for name, seed in (("scan_a", 3), ("scan_b", 4)):
        sc = synth.make_scene(240, 180, 2, seed=seed)
        HS.write_dense_folder(sc, str(root / name), ext=".png")
    script = os.path.join(REPO, "apde-mvs_amd", "run_scans.py")
    out = subprocess.run([sys.executable, script, "--data_dir", str(root), "--no_sam", "--memory_cache", "--flush",
                          "--APD_path", APD_BIN], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    for name in ("scan_a", "scan_b"):
        assert os.path.getsize(root / name / "APD" / "APD.ply") > 0
        assert os.path.exists(root / name / "APD" / "00000000" / "depths.bin")
        assert "RunPatchMatch time" in (root / name / "APD" / "log.txt").read_text()


def test_scan_runner_device_resident(scan, engine, tmp_path):
    """scan_runner.py with the scan's state resident in HBM (torch tensors on cuda:0, device pointers
    through apd_set_problem / apd_get_results, prior resizes as device index gathers): one rank, its
    files equal the Jacobi schedule restated on the host (the same data as the apd binary's
    --ordering jacobi) bit for bit."""
    import shutil
    import sys
    sys.path.insert(0, os.path.join(REPO, "apde-mvs_amd"))
    import scan_runner as SR
    folder = str(tmp_path / "run")
    shutil.copytree(scan, folder)
    SR.run_scan(folder, SR.hip_run_fn(0, on_device=True), 0, 1, None, device="cuda:0")
    expected = HS.run_schedule(folder, run_engine(engine), ordering="jacobi")
    check_outputs(folder, expected)


def test_scan_runner_two_ranks_device_resident(scan, engine, tmp_path):
    """Two scan_runner.py ranks (torch.distributed.run, both on GPU 0, states exchanged as device tensors
    through gloo: RCCL refuses two ranks on one GPU) with the scan resident in HBM: the dynamic queue
    splits every pass's views between the ranks, each problem's inputs are fresh torch / collective
    outputs on the device (the library's stream waits for torch's), and the files equal the Jacobi
    schedule restated on the host bit for bit."""
    import shutil
    import socket
    import sys
    folder = str(tmp_path / "run")
    shutil.copytree(scan, folder)
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    env = dict(os.environ, APD_SCAN_BACKEND="gloo", APD_SCAN_DEVICES="1")
    script = os.path.join(REPO, "apde-mvs_amd", "scan_runner.py")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), script, "--dense_folder", folder],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    expected = HS.run_schedule(folder, run_engine(engine), ordering="jacobi")
    check_outputs(folder, expected)
