import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run on the GPU box")


def golden_files(pattern=""):
    return sorted(os.path.join(GOLDEN, f) for f in os.listdir(GOLDEN)
                  if f.endswith(".npz") and pattern in f)


def load_golden(path):
    """Yield (case dict, arrays dict) for every case in one golden file."""
    with np.load(path, allow_pickle=False) as z:
        cases = json.loads(bytes(z["cases_json"]).decode())
        for i, c in enumerate(cases):
            arrs = {k.split("_", 1)[1]: z[k] for k in z.files if k.startswith(f"c{i}_")}
            yield c, arrs


def golden_cases(pattern=""):
    out = []
    for f in golden_files(pattern):
        for c, a in load_golden(f):
            out.append((c, a))
    return out


def half_matrix(case):
    from qldpcsim_amd import codes
    Hx, Hz = codes.load_code(case["code"])
    return Hz if case["half"] == "X" else Hx
