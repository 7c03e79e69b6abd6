"""bench.py's contract on the GPU: one JSON line with the driver's keys, the
roofline and CPU-baseline objects, and the multi-rank path (launched as the
driver does, torch.distributed.run; here 2 ranks share the one GPU over gloo,
QLDPC_BENCH_BACKEND — on the 8-GPU node it is RCCL, one rank per GPU)."""
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


def test_bench_single_gpu_line():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--batch", "65536",
                        "--cpu-seconds", "1"], cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert KEYS <= set(d) and d["n_gpus"] == 1 and d["value"] > 0
    assert d["roofline"]["bound"] == "hbm" and d["roofline"]["peak"] == 8000.0
    assert d["cpu_baseline"]["kind"] == "port" and d["cpu_baseline"]["value"] > 0
    assert d["config"]["avg_iterations"] == 50.0


def test_bench_two_ranks_share_gpu_over_gloo():
    env = dict(os.environ, QLDPC_BENCH_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29531", "bench.py", "--gpus", "2",
                        "--steps", "1", "--warmup", "1", "--batch", "16384"],
                       cwd=ROOT, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * 16384
    assert "cpu_baseline" not in d and d["value"] > 0
