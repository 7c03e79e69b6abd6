"""Pin the CPU oracle against golden vectors from the unmodified reference.

MS: hard decisions, iteration counts and float64 posteriors bit-exact
(SURVEY.md App. A.1). BP: hard decisions and iterations exact, posteriors
within 1e-6 relative (glibc tanh/atanh vs NumPy's; App. A.2).
"""
import numpy as np
import pytest

from conftest import golden_cases, half_matrix
from oracle import oracle

CASES = [(c, a) for c, a in golden_cases() if "raises" not in c]


def _id(ca):
    c = ca[0]
    return f"{c['algo']}-{c['code']}-{c['half']}-{c['sched']}-{c['kind']}-p{c['p_phys']}-it{c['max_iter']}-osd{c['osd']}"


@pytest.mark.parametrize("ca", CASES, ids=[_id(x) for x in CASES])
def test_oracle_matches_reference(ca):
    c, a = ca
    H = half_matrix(c)
    e, it, post, flags = oracle.decode_batch(c["algo"], H, a["syn"], c["p_phys"] / 3, c["max_iter"],
                                             a["layer_ptr"], a["layer_rows"], nthreads=2)
    if c["osd"] >= 0:
        conv = np.array([bool(np.all((H.astype(np.int64) @ e[k]) % 2 == a["syn"][k]))
                         for k in range(len(it))])
        for k in range(len(it)):
            if not conv[k]:
                e[k] = oracle.osd_dec(H, e[k].astype(np.int64), a["syn"][k].astype(np.int64),
                                      post[k], c["osd"]).astype(np.uint8)
    np.testing.assert_array_equal(it, a["iters"])
    np.testing.assert_array_equal(e, a["ehat"])
    if c["osd"] >= 0:
        return
    if c["algo"] == "MS":
        np.testing.assert_array_equal(post.view(np.uint64), a["post"].view(np.uint64))
    else:
        np.testing.assert_allclose(post, a["post"], rtol=1e-6, atol=0)
