"""Batch driver over scans: the run.py orchestration (run.py:1-240) for the `apd` binary.

Same command line as run.py (flags, defaults, scan lists, dataset detection from --data_dir, LPT
order by image count, one work slot per (GPU, worker), per-scan APD/log.txt, --resume / --review),
and the same per-scan command it emits (run.py:104-119), so a maintainer can point run.py's
--APD_path at apde-mvs_amd/host/build/apd, or use this file, with identical results. Differences:

  * SAM mask generation (tools/run_SAM.py) is out of scope (a learned model with network
    checkpoints): scans without sa_masks/ run like the reference binary does when the folder is
    missing (it logs "Can't find sa mask folder" and runs without SA).
  * --gpus_per_scan K (new): hand K devices to each scan (`apd --gpus a,b,..`, Jacobi passes
    sharded over the devices), for batches with fewer scans than GPUs.
  * --backup_code is not restated (it copies the reference's CUDA sources).

The image-folder normalisation of scripts/dataset_loader.py (candidates images/, undist/images;
suffix filter; images/ symlink) is restated in `ScanLayout`.
"""
from __future__ import annotations

import argparse
import multiprocessing as mp
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

ETH3D_TRAIN = ['courtyard', 'delivery_area', 'electro', 'facade', 'kicker', 'meadow', 'office', 'pipes',
               'playground', 'relief', 'relief_2', 'terrace', 'terrains']
ETH3D_TEST = ['botanical_garden', 'boulders', 'bridge', 'door', 'exhibition_hall', 'lecture_room', 'living_room',
              'lounge', 'observatory', 'old_computer', 'statue', 'terrace_2']
TAT_INTERMEDIATE = ['Family', 'Francis', 'Horse', 'Lighthouse', 'M60', 'Panther', 'Playground']
TAT_ADVANCED = ['Auditorium', 'Ballroom', 'Courtroom', 'Museum', 'Palace', 'Temple']


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--data_dir', type=str, default='/home/ubuntu/Data/DTU/test')
    p.add_argument('--APD_path', type=str, default=os.path.join(HERE, 'host', 'build', 'apd'))
    p.add_argument('--resume', action='store_true', default=False)
    p.add_argument('--gpu_num', type=int, default=1)
    p.add_argument('--work_num', type=int, default=1)
    p.add_argument('--gpus_per_scan', type=int, default=1)
    p.add_argument('--scans', type=str, nargs='+', default=[])
    for flag in ('only_fuse', 'no_fuse', 'memory_cache', 'no_sam', 'no_impetus', 'no_weak_filter', 'no_color',
                 'flush', 'ETH3D_train', 'ETH3D_test', 'TaT_intermediate', 'TaT_advanced', 'export_anchor',
                 'export_curve', 'no_image_symlink', 'review'):
        p.add_argument('--' + flag, action='store_true', default=False)
    p.add_argument('--image_dir_name', type=str, nargs='+', default=['images', 'undist/images'])
    p.add_argument('--image_suffixes', type=str, nargs='+', default=['.jpg', '.jpeg', '.png'])
    return p.parse_args(argv)


class ScanLayout:
    """scripts/dataset_loader.py: SceneDatasetLoader with DatasetLayoutConfig (target images/)."""

    def __init__(self, scan_dir, candidates, suffixes, create_symlink):
        self.scan_dir = os.path.abspath(scan_dir)
        self.candidates = candidates
        self.suffixes = [s.lower() if s.startswith('.') else '.' + s.lower() for s in suffixes if s]
        self.create_symlink = create_symlink

    def image_dir(self):
        for cand in self.candidates:
            path = os.path.join(self.scan_dir, *[c for c in cand.split('/') if c])
            if os.path.isdir(path):
                return path
        raise FileNotFoundError(f'no image directory among {self.candidates} in {self.scan_dir}')

    def ensure_standard_image_dir(self):
        src = self.image_dir()
        canonical = os.path.join(self.scan_dir, 'images')
        if os.path.isdir(canonical):
            return canonical
        if os.path.exists(canonical):
            raise FileExistsError(f'{canonical} exists and is not a directory')
        if not self.create_symlink:
            raise FileNotFoundError(f'{canonical} is missing and symlink creation is disabled')
        os.symlink(src, canonical)
        return canonical

    def count_images(self):
        d = self.image_dir()
        return sum(1 for e in os.listdir(d)
                   if os.path.isfile(os.path.join(d, e)) and os.path.splitext(e)[1].lower() in self.suffixes)


def dataset_of(data_dir, scan):
    """run.py:83-93"""
    if data_dir.find('DTU') != -1:
        return 'DTU'
    if data_dir.find('TaT') != -1:
        return 'TaT_a' if scan in TAT_ADVANCED else 'TaT_i'
    if data_dir.find('ETH3D') != -1:
        return 'ETH3D'
    return 'General'


def apd_command(args, scan_dir, gpus, dataset):
    """The per-scan command of run.py:104-119 (`--gpus` added when a scan gets several devices)."""
    tf = lambda b: 'true' if b else 'false'
    cmd = ('{} --dense_folder {} --gpu_index {} --dataset {} '
           '--only_fuse {} --no_fuse {}  --use_sa {} --memory_cache {} --flush {} '
           '--export_anchor {} --export_curve {} --export_color {} --use_impetus {} --weak_filter {}').format(
        args.APD_path, scan_dir, gpus[0], dataset, tf(args.only_fuse), tf(args.no_fuse), tf(not args.no_sam),
        tf(args.memory_cache), tf(args.flush), tf(args.export_anchor), tf(args.export_curve), tf(not args.no_color),
        tf(not args.no_impetus), tf(not args.no_weak_filter))
    if len(gpus) > 1:
        cmd += ' --gpus {} --ordering jacobi'.format(','.join(str(g) for g in gpus))
    return cmd


_slots = None
_lock = None


def _init(slots, lock):
    global _slots, _lock
    _slots, _lock = slots, lock


def worker(args, scan):
    scan_dir = os.path.join(args.data_dir, scan)
    if not os.path.isdir(scan_dir):
        print('{} is not a dir'.format(scan_dir), flush=True)
        return 1
    try:
        ScanLayout(scan_dir, args.image_dir_name, args.image_suffixes, not args.no_image_symlink).ensure_standard_image_dir()
    except (FileNotFoundError, FileExistsError) as exc:
        print('[{}] cannot prepare the image directory: {}'.format(scan, exc), flush=True)
        return 1
    with _lock:  # acquire a work slot (run.py:73-80)
        pos = next(j for j in range(len(_slots)) if _slots[j] == 0)
        _slots[pos] = 1
    try:
        k = max(1, args.gpus_per_scan)
        first = (pos // args.work_num) * k
        gpus = list(range(first, first + k))
        if not args.no_sam and not os.path.isdir(os.path.join(scan_dir, 'sa_masks')):
            print('[{}] no sa_masks/ (SAM generation is out of scope): running without SA masks'.format(scan), flush=True)
        apd_dir = os.path.join(scan_dir, 'APD')
        os.makedirs(apd_dir, exist_ok=True)
        cmd = apd_command(args, scan_dir, gpus, dataset_of(args.data_dir, scan))
        log_path = os.path.join(apd_dir, 'log.txt')
        cmd += (' >> ' if os.path.exists(log_path) else ' > ') + log_path
        if args.resume and os.path.exists(os.path.join(apd_dir, 'APD.ply')):
            print('APD result exists for {}'.format(scan_dir), flush=True)
            return 0
        print(cmd, flush=True)
        if args.review:
            return 0
        return subprocess.run(cmd, shell=True).returncode
    finally:
        with _lock:
            _slots[pos] = 0


def scan_list(args):
    if args.ETH3D_train:
        return list(ETH3D_TRAIN)
    if args.ETH3D_test:
        return list(ETH3D_TEST)
    if args.TaT_intermediate:
        return list(TAT_INTERMEDIATE)
    if args.TaT_advanced:
        return list(TAT_ADVANCED)
    return list(args.scans) if args.scans else sorted(os.listdir(args.data_dir))


def main(argv=None):
    args = parse_args(argv)
    print(args, flush=True)
    scans = []
    for scan in scan_list(args):
        scan_dir = os.path.join(args.data_dir, scan)
        if not os.path.isdir(scan_dir):
            print('{} is not a dir'.format(scan_dir), flush=True)
            continue
        lay = ScanLayout(scan_dir, args.image_dir_name, args.image_suffixes, not args.no_image_symlink)
        try:
            if not args.no_image_symlink:
                lay.ensure_standard_image_dir()
            scans.append((scan, lay.count_images()))
        except (FileNotFoundError, FileExistsError) as exc:
            print('skipping {}: {}'.format(scan_dir, exc), flush=True)
    if not scans:
        print('No valid scans found.', flush=True)
        return 0
    scans.sort(key=lambda s: -s[1])  # largest first (run.py:214)
    names = [s for s, _ in scans]
    print('scans: {}'.format(names), flush=True)
    slots_n = min(args.work_num * max(1, args.gpu_num // max(1, args.gpus_per_scan)), len(names))
    slots, lock = mp.Array('i', [0] * slots_n), mp.Lock()
    with mp.Pool(processes=slots_n, initializer=_init, initargs=(slots, lock)) as pool:
        codes = [pool.apply_async(worker, (args, s)) for s in names]
        rc = [c.get() for c in codes]
    print('done', flush=True)
    return 0 if all(r == 0 for r in rc) else 1


if __name__ == '__main__':
    sys.exit(main())
