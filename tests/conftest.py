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


@pytest.fixture
def qopt():
    """Set library options (qldpc_set_option) for one test: qopt(force_hbm=1, ...);
    every option touched gets its previous value back afterwards."""
    from qldpcsim_amd import _lib
    saved = {}

    def set_(**kw):
        for k, v in kw.items():
            saved.setdefault(k, _lib.get_option(k))
            _lib.set_option(k, v)
    yield set_
    for k, v in saved.items():
        _lib.set_option(k, v)


@pytest.fixture
def osdpol():
    """Set the OSD reliability-order policy (decoders.OSD_POLICY) for one test."""
    from qldpcsim_amd import decoders
    old = dict(decoders.OSD_POLICY)
    yield decoders.set_osd_policy
    decoders.OSD_POLICY.update(old)


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
