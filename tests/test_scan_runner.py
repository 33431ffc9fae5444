"""CPU (gloo, world_size 2): the view-sharded scan runner (apde-mvs_amd/scan_runner.py).

Two ranks each process half of the views of every pass and exchange the new depth maps with one
torch.distributed all-gather per pass. The files they write must equal, bit for bit, the Jacobi
schedule restated in tests/host_schedule.py on one process -- with the CPU oracle standing in for the
HIP engine (test infrastructure; the runner itself only takes a run_fn). A 1-rank run must give the
same files, i.e. the result does not depend on the number of ranks.
"""
import os
import shutil

import numpy as np
import pytest
import torch.multiprocessing as mp

import host_schedule as HS
import oracle_lib
import synth


def _oracle_fn():
    lib = oracle_lib.load()
    return lambda arr: oracle_lib.run(lib, arr, nthreads=2)


def _rank_main(rank, world, folder, port, slow_rank=-1, log=None):
    import sys
    import time
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "apde-mvs_amd")]
    import torch.distributed as dist
    import scan_runner as SR
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fn = _oracle_fn()

    def run_fn(arr):
        if rank == slow_rank:
            time.sleep(2.0)
        if log:
            with open(f"{log}.{rank}", "a") as fh:
                fh.write(f"{arr.seed}\n")
        return fn(arr)
    SR.run_scan(folder, run_fn, rank, world, SR.Exchange(world, rank, None))
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def scan(tmp_path_factory):
    sc = synth.make_scene(128, 96, 3, seed=11)
    folder = str(tmp_path_factory.mktemp("scan"))
    HS.write_dense_folder(sc, folder, ext=".png", masks=True)
    expected = HS.run_schedule(folder, _oracle_fn(), ordering="jacobi")
    return folder, expected


def _check(folder, expected):
    for ref, exp in expected.items():
        d = os.path.join(folder, "APD", f"{ref:08d}")
        for name, key in (("depths.bin", "depth"), ("normals.bin", "normal"), ("weak.bin", "weak"),
                          ("confidence.bin", "conf")):
            got = synth.read_bin_mat(os.path.join(d, name))
            e = exp[key]
            if e.dtype == np.float32:
                assert np.array_equal(got.view(np.uint32), e.view(np.uint32)), (ref, name)
            else:
                assert np.array_equal(got, e), (ref, name)


def test_two_ranks_equal_single_process_jacobi(scan, tmp_path):
    folder, expected = scan
    run = str(tmp_path / "run")
    shutil.copytree(folder, run)
    port = 29500 + (os.getpid() % 2000)
    mp.spawn(_rank_main, args=(2, run, port), nprocs=2, join=True)
    _check(run, expected)


def test_one_rank_equals_jacobi(scan, tmp_path):
    import scan_runner as SR
    folder, expected = scan
    run = str(tmp_path / "run")
    shutil.copytree(folder, run)
    SR.run_scan(run, _oracle_fn(), 0, 1, None)
    _check(run, expected)


def test_runner_matches_restated_host_io(scan):
    """The runner's C++-backed decode/resize/camera path agrees with the Python restatement."""
    import scan_runner as SR
    folder, _ = scan
    host = SR.HostLib()
    img = host.read_gray(os.path.join(folder, "images", "00000000.png")).astype(np.float32)
    from PIL import Image
    assert np.array_equal(img, np.asarray(Image.open(os.path.join(folder, "images", "00000000.png")), np.float32))
    assert np.array_equal(host.resize_linear(img, 64, 48), HS.resize_linear(img, 64, 48))
    cam = host.read_camera(os.path.join(folder, "cams", "00000001_cam.txt"))
    exp = HS.read_cam(os.path.join(folder, "cams", "00000001_cam.txt"))
    for k in ("K", "R", "t", "c"):
        assert np.array_equal(cam[k], exp[k])


def test_dynamic_queue_balances_a_slow_rank(scan, tmp_path):
    """The views of a pass come from a dynamic queue: with rank 0 slowed down, rank 1 takes more of
    them, every (view, pass) is processed exactly once, and the files still equal the Jacobi schedule."""
    folder, expected = scan
    run = str(tmp_path / "run")
    shutil.copytree(folder, run)
    log = str(tmp_path / "seeds")
    port = 31500 + (os.getpid() % 2000)
    mp.spawn(_rank_main, args=(2, run, port, 0, log), nprocs=2, join=True)
    _check(run, expected)
    seeds = [open(f"{log}.{r}").read().split() for r in (0, 1)]
    assert len(seeds[1]) > len(seeds[0])
    allseeds = seeds[0] + seeds[1]
    assert len(allseeds) == len(set(allseeds))  # seed = f(view, pass): no view ran twice in a pass
    n_views = len(expected)
    assert len(allseeds) % n_views == 0


def test_nearest_index_equals_host_resize():
    """The runner's INTER_NEAREST index gather == the C++ host resize (host/image.cpp) on an index map."""
    import scan_runner as SR
    host = SR.HostLib()
    for (sw, sh, dw, dh) in [(96, 72, 48, 36), (50, 37, 100, 75), (61, 43, 33, 91), (31, 17, 31, 17)]:
        idx = np.arange(sw * sh, dtype=np.int32).reshape(sh, sw)
        ref = host.resize_nearest(idx, dw, dh)
        yo, xo = SR.nearest_index(sw, sh, dw, dh)
        assert np.array_equal(idx[yo][:, xo], ref)


def test_wire_format_round_trip():
    """The exchange's 18 B/px wire format (scan_runner.wire_pack): bit-identical round trip of a
    [6, h, w] state whose planes 4-5 hold u8 values, at odd sizes and as the k-th row of a [k, bytes]
    gather buffer (16-byte row padding keeps the f32 view aligned)."""
    import sys
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "apde-mvs_amd"))
    import scan_runner as SR
    g = torch.Generator().manual_seed(5)
    for h, w in [(5, 7), (1, 1), (33, 17), (64, 48)]:
        st = torch.randn(6, h, w, generator=g)
        st[0, 0, 0] = float("nan")
        st[1, -1, -1] = -0.0
        st[4] = torch.randint(0, 3, (h, w), generator=g).float()
        st[5] = torch.randint(0, 256, (h, w), generator=g).float()
        assert SR.wire_bytes(h, w) % 16 == 0 and SR.wire_bytes(h, w) >= 18 * h * w
        buf = torch.stack([SR.wire_pack(st * 0), SR.wire_pack(st), SR.wire_pack(st)])
        for k in (1, 2):
            back = SR.wire_unpack(buf[k], h, w)
            assert torch.equal(back.view(torch.int32), st.view(torch.int32))
