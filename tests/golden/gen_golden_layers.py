"""Pin the layer schedules to the reference's own `layerize` and schedule
selection (simulator.py:212-236), not to a restatement.

Build container only. `qLDPCsim/simulator.py` does not import on Python 3.10
(a syntax error at :347) and needs Stim, so the generator reads the file as
text, cuts out the nested `def layerize` (:212-224) and the `match
decSchedule` block that builds layersX / layersZ (:228-236), dedents both and
executes them unchanged with each bundled (Hx, Hz) in scope. The layers the
reference builds are stored as data (tests/golden/schedules/layers.npz): per code and
schedule in {L, S}, layersX (built from Hx, used by the reference with Hz,
:278-282) and layersZ, each as (ptr, rows).

Usage: python tests/golden/gen_golden_layers.py
"""
import json
import os
import sys
import textwrap

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from qldpcsim_amd import codes  # noqa: E402  (bundled matrices only)

REF = "/root/reference/qLDPCsim/simulator.py"


def reference_block():
    """Source text of simulator.py's layerize + schedule selection, dedented."""
    lines = open(REF).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.strip().startswith("def layerize("))
    stop = next(i for i, l in enumerate(lines) if i > start and l.strip().startswith("decFailuresX"))
    src = textwrap.dedent("\n".join(lines[start:stop]))
    assert "case \"L\" | \"S\":" in src and "layersZ = layerize(Hz" in src, "unexpected reference layout"
    return src, start + 1, stop


def main():
    src, first, last = reference_block()
    code = compile(src, f"{REF}:{first}-{last}", "exec")
    out, index = {}, []
    for name in codes.available():
        Hx, Hz = codes.load_code(name)
        for sched in ("L", "S"):
            env = {"np": np, "Hx": Hx, "Hz": Hz, "decSchedule": sched,
                   "m_x": Hx.shape[0] if Hx.size else 0, "m_z": Hz.shape[0] if Hz.size else 0}
            exec(code, env)
            for half in ("X", "Z"):
                layers = env[f"layers{half}"]
                sizes = [len(l) for l in layers]
                ptr = np.zeros(len(layers) + 1, dtype=np.int32)
                ptr[1:] = np.cumsum(sizes)
                rows = np.concatenate([np.asarray(l, dtype=np.int64) for l in layers]).astype(np.int32)
                key = f"{name}__{sched}__{half}"
                out[key + "__ptr"], out[key + "__rows"] = ptr, rows
                index.append(key)
    out["index_json"] = np.frombuffer(json.dumps({"source": f"{REF}:{first}-{last}", "keys": index}).encode(),
                                      dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "schedules", "layers.npz"), **out)
    print(f"{len(index)} layer lists from {REF}:{first}-{last}")


if __name__ == "__main__":
    main()
