"""The ctypes binding shown in INTEGRATION.md §2 works as written (GPU)."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_integration_md_ctypes_stub_decodes_like_the_oracle():
    import qldpcsim_amd._lib  # noqa: F401  (loads torch's HIP runtime first, as the package does)
    from oracle import oracle
    from qldpcsim_amd import _lib, codes
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = re.findall(r"```python\n(import ctypes.*?)```", txt, re.S)[0]
    block = block.replace("/path/to/qldpcsim_amd/_build/libqldpc_hip.so", _lib.LIB_PATH)
    ns = {}
    exec(block, ns)
    Hx, Hz = codes.load_code("LP04_0")
    rng = np.random.default_rng(4)
    syn = rng.integers(0, 2, (4, Hz.shape[0])).astype(np.uint8)
    e, it, _, _ = oracle.decode_batch("MS", Hz, syn, 0.01, 20)
    for k in range(4):
        ek, ik = ns["MS_decoder_gpu"](Hz, syn[k], 0.01, max_iter=20)
        assert ik == it[k]
        np.testing.assert_array_equal(ek.astype(np.uint8), e[k])
