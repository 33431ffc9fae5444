"""run_scans.py == run.py's orchestration (run.py:1-240), checked in --review mode (commands printed,
nothing executed): scan discovery, image-folder normalisation (dataset_loader.py), LPT order by image
count, dataset detection from --data_dir, GPU slots, and the exact per-scan command line."""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(REPO, "apde-mvs_amd", "run_scans.py")


def make_scan(root, name, n_images, subdir="images", ext=".jpg"):
    d = os.path.join(root, name, *subdir.split("/"))
    os.makedirs(d)
    for i in range(n_images):
        open(os.path.join(d, f"{i:08d}{ext}"), "wb").close()
    open(os.path.join(d, "notes.txt"), "w").close()  # filtered out by the suffix list


def run(args):
    out = subprocess.run([sys.executable, SCRIPT] + args, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    return out.stdout


def test_review_mode_commands(tmp_path):
    root = tmp_path / "ETH3D"
    root.mkdir()
    make_scan(str(root), "office", 3)
    make_scan(str(root), "pipes", 5, subdir="undist/images", ext=".JPG")
    (root / "README").write_text("not a scan")
    make_scan(str(root), "empty_scan", 0, subdir="other")
    stdout = run(["--data_dir", str(root), "--gpu_num", "2", "--review", "--APD_path", "/opt/apd"])
    cmds = [l for l in stdout.splitlines() if l.startswith("/opt/apd ")]
    # largest scan first (the submission order; the two slots then run concurrently); empty_scan has
    # no image folder among the candidates and is skipped
    assert "scans: ['pipes', 'office']" in stdout
    assert sorted(re.search(r"--dense_folder (\S+)", c).group(1) for c in cmds) == [str(root / "office"), str(root / "pipes")]
    assert os.path.islink(root / "pipes" / "images")  # images/ -> undist/images
    for c in cmds:
        assert re.search(r"--gpu_index [01] ", c)
        assert ("--dataset ETH3D --only_fuse false --no_fuse false  --use_sa true --memory_cache false "
                "--flush false --export_anchor false --export_curve false --export_color true "
                "--use_impetus true --weak_filter true") in c
        assert re.search(r" > \S+/APD/log\.txt$", c)


def test_flags_and_multi_gpu_scans(tmp_path):
    root = tmp_path / "TaT"
    root.mkdir()
    make_scan(str(root), "Family", 4)
    make_scan(str(root), "Palace", 2)
    stdout = run(["--data_dir", str(root), "--gpu_num", "4", "--gpus_per_scan", "2", "--review", "--no_sam",
                  "--memory_cache", "--no_fuse", "--APD_path", "apd"])
    cmds = {re.search(r"--dense_folder \S+/(\w+) ", l).group(1): l for l in stdout.splitlines() if l.startswith("apd ")}
    assert "--dataset TaT_i" in cmds["Family"] and "--dataset TaT_a" in cmds["Palace"]
    for c in cmds.values():
        assert "--use_sa false" in c and "--memory_cache true" in c and "--no_fuse true" in c
        g = re.search(r"--gpus (\d),(\d) --ordering jacobi", c)
        assert g and int(g.group(2)) == int(g.group(1)) + 1
