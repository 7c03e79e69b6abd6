"""bench.py host logic without a GPU: argument contract, the algorithmic
byte model (SURVEY.md §8d table values), host core detection, the device-code
hash the roofline profile is keyed on, and the loud failures."""
import os
import subprocess
import sys

import numpy as np

from conftest import ROOT

import bench
from qldpcsim_amd import codes, schedule


def test_algorithmic_bytes_match_survey_table():
    # MS-F B_it per half, MS-L B/iter for X + Z
    for code, bit, layered in (("LP118_0", 27392, 110464), ("LP04_0", 8456, 32312), ("LP118_2", 51360, 207120)):
        Hx, Hz = codes.load_code(code)
        lp, lr = schedule.pack_layers(None, Hz.shape[0])
        assert bench.algorithmic_bytes_per_iter(Hz.astype(np.int64), lp, lr, 4) == bit
        lx, lz = schedule.select_layers(Hx, Hz, "L")
        tot = sum(bench.algorithmic_bytes_per_iter(H.astype(np.int64), *schedule.pack_layers(l, H.shape[0]), 4)
                  for H, l in ((Hz, lx), (Hx, lz)))
        assert tot == layered


def test_host_cores_and_device_code_hash():
    n, how = bench.host_cores()
    assert 1 <= n <= (os.cpu_count() or 1) and how
    from qldpcsim_amd import _lib
    h = bench.device_code_sha(_lib.LIB_PATH)
    assert len(h) == 64 and h == bench.device_code_sha(_lib.LIB_PATH)


def test_gpus_disagreeing_with_world_size_fails():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "3"], cwd=ROOT, capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode != 0 and "disagrees with WORLD_SIZE" in r.stderr


def test_more_ranks_than_devices_fails_loudly():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("QLDPC_BENCH_BACKEND", None)
    import torch
    n = torch.cuda.device_count()
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n + 2)], cwd=ROOT, capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode != 0 and "HIP device(s) visible" in r.stderr


def test_no_device_fails_loudly():
    if __import__("torch").cuda.device_count():
        return
    r = subprocess.run([sys.executable, "bench.py", "--cpu-seconds", "0"], cwd=ROOT, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "no HIP device" in r.stderr
