"""Check-node schedules (layer partitions) — host-side precompute.

Restates `simulate_p`'s nested `layerize` (reference simulator.py:212-224)
and its schedule selection with the reference's cross-wiring
(simulator.py:228-236, used at :278-282): the X-half decoder runs on Hz but
receives the layers computed from Hx, and vice versa.
Layers are handed to the decoder as explicit row lists (CSR-style
`layer_ptr` / `layer_rows`), never re-derived from the matrix being decoded.
"""
import numpy as np


def layerize(H: np.ndarray, serial: bool = False) -> list:
    """Greedy partition of consecutive rows into column-disjoint windows.

    Same loop as simulator.py:212-224: grow the window [mDn, mUp) while no
    column of H[mDn:mUp] has weight > 1 (and, when `serial`, while the window
    holds at most one row); emit it; restart at the row that broke it. The
    final `append` happens even when it yields an empty range (m == 0).
    """
    layers = []
    m = H.shape[0]
    mUp = 1
    mDn = 0
    while mUp <= m:
        if np.max(np.sum(H[mDn:mUp, :], axis=0)) > 1 or (serial and mUp > mDn + 1):
            layers.append(np.arange(mDn, mUp - 1))
            mDn = mUp - 1
        else:
            mUp += 1
    layers.append(np.arange(mDn, mUp - 1))
    return layers


def select_layers(Hx: np.ndarray, Hz: np.ndarray, decSchedule: str):
    """Return (layersX, layersZ) exactly as simulator.py:228-236 builds them.

    layersX is later used with Hz (X half) and layersZ with Hx (Z half).
    """
    m_x = Hx.shape[0] if Hx.size else 0
    m_z = Hz.shape[0] if Hz.size else 0
    if decSchedule == "F":
        return [np.arange(m_x)], [np.arange(m_z)]
    if decSchedule in ("L", "S"):
        serial = decSchedule == "S"
        return layerize(Hx, serial=serial), layerize(Hz, serial=serial)
    raise ValueError("Unrecognized decoder scheduling option.")


def pack_layers(layers, m: int):
    """Flatten a list of row arrays into (layer_ptr int32[L+1], layer_rows int32[sum])."""
    if layers is None:
        layers = [np.arange(m)]
    sizes = [len(np.asarray(l).reshape(-1)) for l in layers]
    ptr = np.zeros(len(layers) + 1, dtype=np.int32)
    ptr[1:] = np.cumsum(sizes, dtype=np.int64)
    rows = (np.concatenate([np.asarray(l, dtype=np.int64).reshape(-1) for l in layers])
            if layers else np.zeros(0, dtype=np.int64))
    if rows.size and (rows.min() < 0 or rows.max() >= m):
        # the reference raises IndexError on out-of-range layer rows (decoders.py:156)
        raise IndexError(f"layer row index out of range for a matrix with {m} rows")
    return ptr, rows.astype(np.int32)
