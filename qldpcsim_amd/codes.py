"""Bundled CSS code pairs (Hx, Hz).

The matrices are the reference's shipped PCM data (`data/*.npy`, SURVEY.md §2
row 14) plus `PCMlibrary.bicycle_code()` (PCMlibrary.py:66-78), bit-packed by
`tools/import_pcm_data.py`. Returned exactly as the reference's
`load_matrix` returns them: `(mat % 2).astype(np.int8)` (simulator.py:35).
"""
import os
from functools import lru_cache

import numpy as np

_DATA = os.path.join(os.path.dirname(__file__), "data", "pcm_library.npz")


@lru_cache(maxsize=1)
def _library():
    with np.load(_DATA, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def available():
    return sorted({k.split("__")[0] for k in _library()})


def load_pcm(name: str, which: str) -> np.ndarray:
    """Return one parity-check matrix (`which` in {"Hx", "Hz"}) as int8."""
    lib = _library()
    key = f"{name}__{which}"
    if key not in lib:
        raise ValueError(f"unknown code {name!r} (available: {available()})")
    m, n = (int(v) for v in lib[key + "__shape"])
    return np.unpackbits(lib[key], axis=1, count=n)[:m].astype(np.int8)


def load_code(name: str):
    """Return (Hx, Hz) for a bundled code, e.g. "LP118_0"."""
    return load_pcm(name, "Hx"), load_pcm(name, "Hz")
