"""bench.py's contract on the GPU: one JSON line with the driver's keys, the
roofline (on-chip bound priced from the committed counter profile) and
CPU-baseline objects, and the multi-rank paths: spawned by `--gpus N` itself,
and launched by torch.distributed.run as the driver does. On this one-GPU box
two ranks share the device over gloo (QLDPC_BENCH_BACKEND); with RCCL,
`--gpus 2` must refuse to run."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config", "roofline"}


def _last_json(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


def _bench(*args, env=None, timeout=110):
    return subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, capture_output=True, text=True,
                          timeout=timeout, env=env)


def test_bench_single_gpu_line():
    r = _bench("--steps", "2", "--warmup", "1", "--batch", "65536", "--cpu-seconds", "1", "--sim-shots", "65536")
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    sim = d["simulate"]                                        # the configs[3] / configs[4] legs
    c3, c4 = sim["configs3"], sim["configs4"]
    assert c3["shots"] == 65536 and c3["value"] > 0 and c3["scaling"] == "strong"
    assert c3["weak_per_rank"]["scaling"] == "weak" and c3["weak_per_rank"]["value"] == c3["value"]
    assert c3["osd_shots"] > 0 and c3["host_order_shots"] == 0   # NumPy's order on the device
    assert 0.5 < c3["qBLER"] < 1.0
    # configs[4]: the four-point curve through simulate's p loop; the qBLER
    # rises with p, and BP never gets OSD from simulate (simulator.py:281-282)
    assert [pt["p"] for pt in c4["curve"]] == [0.01, 0.02, 0.05, 0.1]
    assert all(pt["shots"] == 65536 and pt["value"] > 0 for pt in c4["curve"])
    q = [pt["qBLER"] for pt in c4["curve"]]
    assert q == sorted(q) and q[-1] > 0.1
    assert d["parity_pin"]["order"] and d["parity_pin"]["libm"]
    assert KEYS <= set(d) and d["n_gpus"] == 1 and d["value"] > 0
    rf = d["roofline"]
    assert rf["kernel"] == "ms_flood_kernel<8, 4>"
    assert rf["hbm"]["algorithmic_gbs"] > 0 and rf["hbm"]["peak_gbs"] == 8000.0
    if rf["profile"] is not None:                  # committed profile of this build
        assert rf["bound"] in ("valu", "lds") and 0.05 < rf["frac"] <= 1.05
        assert 0 < rf["hbm"]["frac"] < 1 and rf["traffic"] > 0
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1
    assert [l["sample"].split("oracle/")[1].split()[0] for l in cb["legs"]] == \
        ["qldpc_oracle.c,", "numpy_dense.py"]
    assert cb["reference_context"]["value"] == 2.61
    assert d["config"]["avg_iterations"] == 50.0
    hs = d["hbm_streaming"]                         # the same workload on the HBM-resident kernel
    assert hs["kernel"].startswith("hbm_tile_kernel<0, 8") and hs["value"] > 0
    assert 0 < hs["frac"] < 1 and hs["peak_gbs"] == 8000.0


def test_bench_hbm_path_line():
    """--path hbm times the HBM-resident kernel as the main leg: same workload,
    its roofline includes the measured-HBM unit (bound hbm when the committed
    profile matches this build)."""
    r = _bench("--path", "hbm", "--steps", "1", "--warmup", "1", "--batch", "65536", "--cpu-seconds", "0",
               "--sim-legs", "")
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    rf = d["roofline"]
    assert rf["kernel"] == "hbm_tile_kernel<0, 8, 4>" and d["config"]["avg_iterations"] == 50.0
    assert "hbm_streaming" not in d
    if rf["profile"] is not None:
        assert set(rf["units"]) == {"valu", "lds", "hbm"} and rf["bound"] == "hbm"
        assert 0.05 < rf["frac"] <= 1.05


def test_bench_layered_channel_line():
    r = _bench("--steps", "1", "--warmup", "1", "--batch", "16384", "--cpu-seconds", "0",
               "--code", "LP118_2", "--schedule", "L", "--p", "0.05", "--sim-legs", "")
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["roofline"]["kernel"].startswith("ms_layered_kernel<8")
    assert 1.0 < d["config"]["avg_iterations"] < 10.0


def test_bench_spawns_ranks_itself_over_gloo():
    env = dict(os.environ, QLDPC_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = _bench("--gpus", "2", "--steps", "1", "--warmup", "1", "--batch", "16384", "--sim-legs", "3",
               "--sim-shots", "32768", env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * 16384
    assert "cpu_baseline" not in d and d["value"] > 0
    leg = d["simulate"]["configs3"]                           # a fixed total, each rank its share
    assert leg["n_ranks"] == 2 and leg["shots"] == 32768 and len(leg["per_rank"]) == 2
    assert [r["shots"] for r in leg["per_rank"]] == [16384, 16384]
    c = leg["counters"]
    assert 0 < c["decSuccessExact"] + c["decSuccessDegen"] < leg["shots"] and leg["host_order_shots"] == 0
    weak = leg["weak_per_rank"]                               # 32768 per rank
    assert weak["shots"] == 2 * 32768 and weak["scaling"] == "weak"
    assert "configs4" not in d["simulate"]


def test_bench_refuses_more_ranks_than_gpus_over_rccl():
    env = dict(os.environ)
    env.pop("QLDPC_BENCH_BACKEND", None)
    env.pop("WORLD_SIZE", None)
    import torch
    n = torch.cuda.device_count()
    r = _bench("--gpus", str(n + 1), "--steps", "1", "--warmup", "0", "--batch", "1024", "--sim-legs", "", env=env)
    assert r.returncode != 0 and "HIP device(s) visible" in r.stderr


def test_bench_two_ranks_share_gpu_over_gloo_torchrun():
    env = dict(os.environ, QLDPC_BENCH_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29531", "bench.py", "--gpus", "2",
                        "--steps", "1", "--warmup", "1", "--batch", "16384", "--sim-legs", "3", "--sim-shots",
                        "16384"],
                       cwd=ROOT, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * 16384
    assert "cpu_baseline" not in d and d["value"] > 0
