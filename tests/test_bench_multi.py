"""bench.py's multi-GPU launch: `python3 bench.py --gpus N` starts its own N ranks (torch.distributed.run
on 127.0.0.1, before anything touches the GPU) and the N > 1 line carries the timed per-pass state
exchange (scan_runner.Exchange). CPU tests cover the launch logic; the GPU test runs two ranks
on one GPU through gloo (RCCL refuses two ranks on one device)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_self_launch_cmd():
    assert bench.self_launch_cmd(["--gpus", "1"], 1, {}) is None
    # already a rank of the driver's torch.distributed.run: no second launch
    assert bench.self_launch_cmd(["--gpus", "8"], 8, {"WORLD_SIZE": "8"}) is None
    cmd = bench.self_launch_cmd(["--gpus", "4", "--steps", "3"], 4, {"APD_BENCH_PORT": "29612"})
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29612" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert os.path.samefile(cmd[-5], os.path.join(REPO, "bench.py"))
    free = bench.self_launch_cmd(["--gpus", "2"], 2, {})
    port = int([c for c in free if c.startswith("--master-port=")][0].split("=")[1])
    assert 0 < port < 65536


def test_bench_import_touches_no_gpu_runtime():
    """The parent of the self-launch must not have initialised the GPU before it starts the ranks: importing
    bench (everything main() does before the launch) loads neither torch nor the HIP library."""
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "print('torch' in sys.modules, 'apd_abi' in sys.modules)" % REPO)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["False", "False"]


def test_state_exchange_gloo_cpu():
    """state_exchange over a one-rank gloo group on the CPU: the all-gather returns the state and the timed
    form returns a duration."""
    import torch
    import torch.distributed as tdist
    import socket
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        st = torch.arange(6 * 4 * 8, dtype=torch.float32).reshape(6, 4, 8)
        ex, timed, nbytes = bench.state_exchange(tdist, torch, st, 1, kmax=3)
        assert nbytes == 18 * 4 * 8  # (a multiple of 16 already: no row padding)
        ex(3)
        ex(1)
        assert timed(2, 2) >= 0.0
    finally:
        tdist.destroy_process_group()


@pytest.mark.gpu
def test_bench_two_ranks_self_launch():
    """`bench.py --gpus 2` at 378x252 with both ranks on GPU 0 (gloo): rc 0, one JSON line with
    n_gpus == 2, the per-rank step times and the exchange timing."""
    env = dict(os.environ, APD_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--width", "378",
                        "--height", "252", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--c2", "0",
                        "--rich", "0", "--sa", "0", "--end-to-end", "0"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    mg = line["multi_gpu"]
    assert mg["exchange_ms"] > 0 and len(mg["rank_ms_per_step"]) == 2
    # the 18 B/px wire format (scan_runner.wire_pack), ceil(26 views / 2 ranks) problems per exchange
    assert mg["exchange_bytes_per_rank"] == 18 * 378 * 252 and mg["exchange_bytes_per_px"] == 18
    assert mg["problems_per_rank_per_exchange"] == 13 and mg["exchanges_in_timed_region"] == 1
