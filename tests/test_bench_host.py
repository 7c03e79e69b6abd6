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


def test_kernel_code_hash_keys_committed_profiles():
    """Each roofline profile entry is keyed by its own kernel's machine code:
    the demangler maps the library's symbols to rocprofv3's kernel names, every
    decode kernel bench.py can price has a hash, and distinct kernels differ."""
    from qldpcsim_amd import _lib
    assert bench._demangle_kernel("_ZN5qldpc15ms_flood_kernelILi8ELi4EEEvNS_10DecodeArgsE") == "ms_flood_kernel<8, 4>"
    assert bench._demangle_kernel("_ZN5qldpc14bp_team_kernelILb0ELi8ELi4EEEvNS_10DecodeArgsE") == \
        "bp_team_kernel<false, 8, 4>"
    assert bench._demangle_kernel("_Z3foov") is None
    names = ["ms_flood_kernel<8, 4>", "ms_layered_kernel<8, 1>", "bp_team_kernel<false, 8, 4>",
             "bp_team_lg_kernel<8, 4>", "hbm_tile_kernel<0, 8, 4>", "hbm_tile_kernel<1, 8, 4>",
             "osd_block_kernel<17, 8, 2>"]
    hs = [bench.kernel_code_sha(_lib.LIB_PATH, k) for k in names]
    assert all(h is not None and len(h) == 64 for h in hs) and len(set(hs)) == len(hs)
    assert bench.kernel_code_sha(_lib.LIB_PATH, "no_such_kernel<1>") is None
    # a profile entry is found only under its own hash
    src, ent = bench.find_profile("ms_flood_kernel<8, 4>", None, "0" * 64)
    assert src is None and ent is None


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


def test_find_profile_matches_the_workload(tmp_path, monkeypatch):
    """Two entries of one kernel build (same machine-code hash) profiled on
    different workloads: the roofline takes the counters of its own workload
    (code, decoder, schedule, p, iterations), newest round first whatever the
    tag spelling (r04z < r04aa), and flags a build match of another workload."""
    import json
    d = tmp_path / "profiles"
    d.mkdir()
    ent = lambda args, v: {"kernel": "ms_layered_kernel<8, 1>", "code_sha256": "ab" * 32,  # noqa: E731
                           "bench_args": args, "per_half_shot_iteration": {"valu_insts": v}}
    (d / "r04z_roofline.json").write_text(json.dumps({"kernels": [
        ent("--code LP118_2 --schedule L --p 0.1 --batch 131072", 3.0)]}))
    (d / "r04aa_roofline.json").write_text(json.dumps({"kernels": [
        ent("--code LP118_2 --schedule L --p 0.05 --batch 262144", 1.0),
        ent("--code LP118_2 --schedule L --p 0.1 --batch 131072", 2.0)]}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    w = bench.workload_of(bench.parse(["--code", "LP118_2", "--schedule", "L", "--p", "0.1"]))
    src, k = bench.find_profile("ms_layered_kernel<8, 1>", None, "ab" * 32, w)
    assert src.endswith("r04aa_roofline.json") and k["per_half_shot_iteration"]["valu_insts"] == 2.0
    assert k["workload_match"] is True
    w5 = bench.workload_of(bench.parse(["--code", "LP118_2", "--schedule", "L", "--p", "0.05"]))
    assert bench.find_profile("ms_layered_kernel<8, 1>", None, "ab" * 32, w5)[1]["per_half_shot_iteration"] == \
        {"valu_insts": 1.0}
    wf = bench.workload_of(bench.parse(["--code", "LP118_0"]))
    src, k = bench.find_profile("ms_layered_kernel<8, 1>", None, "ab" * 32, wf)
    assert k["workload_match"] is False
    assert bench.find_profile("ms_layered_kernel<8, 1>", None, "cd" * 32, w) == (None, None)
