"""Pin the dense NumPy restatement (oracle/numpy_dense.py, the CPU-baseline
leg 1 of BASELINE.md) to the golden vectors of the unmodified reference:
MS hard decisions, iteration counts and float64 posteriors bit-exact."""
import numpy as np
import pytest

from conftest import golden_cases, half_matrix
from oracle import numpy_dense

# every MS golden case without OSD; the heavier LP118_2 / bicycle cases only
# at small iteration caps so the CPU suite stays fast
CASES = [(c, a) for c, a in golden_cases("ms_") if "raises" not in c and c["osd"] < 0 and
         (c["code"] not in ("LP118_2", "bicycle") or c["max_iter"] <= 7)]


def _id(ca):
    c = ca[0]
    return f"{c['code']}-{c['half']}-{c['sched']}-{c['kind']}-p{c['p_phys']}-it{c['max_iter']}"


def _layers(a):
    lp, lr = a["layer_ptr"], a["layer_rows"]
    return [lr[lp[i]:lp[i + 1]] for i in range(len(lp) - 1)]


@pytest.mark.parametrize("ca", CASES, ids=[_id(x) for x in CASES])
def test_dense_restatement_matches_reference(ca):
    c, a = ca
    H = half_matrix(c)
    e, it, post = numpy_dense.decode_batch_dense(H, a["syn"], c["p_phys"] / 3, c["max_iter"], _layers(a))
    np.testing.assert_array_equal(it, a["iters"])
    np.testing.assert_array_equal(e, a["ehat"])
    np.testing.assert_array_equal(post.view(np.uint64), a["post"].view(np.uint64))
