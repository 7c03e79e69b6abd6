"""Pin the CPU oracle against golden vectors from the unmodified reference.

MS: hard decisions, iteration counts and float64 posteriors bit-exact
(SURVEY.md App. A.1). BP: hard decisions and iterations exact, posteriors
within 1e-6 relative (glibc tanh/atanh vs NumPy's; App. A.2).
"""
import numpy as np
import pytest

from conftest import golden_cases, half_matrix
from oracle import oracle

CASES = [(c, a) for c, a in golden_cases() if "raises" not in c and c["max_iter"] < 100]
BP100 = golden_cases("_it100")


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


def test_oracle_bp100_against_reference():
    """100-iteration BP golden set (configs[2] LP118_0 F/L, configs[4] LP118_2 L
    p-sweep, 8 shots per p and half, plus never-converging syndromes).

    Decodes that stop within 30 iterations: iterations and hard decisions
    exact, posteriors within the north-star 1e-5 (worst seen 8.4e-6).

    Longer decodes are chaotic: BP at 100 iterations amplifies the last-ULP
    differences between include/qldpc_libm.h and NumPy's tanh / arctanh (SVML
    on this AVX-512 host; glibc on others, so the reference's own output
    depends on the machine it runs on). There, iterations and hard decisions
    agree on 26 of the 28 shots of the set; the test pins that rate (>= 85 %)
    and that no short decode is affected."""
    short = long_ = long_same = 0
    for c, a in BP100:
        H = half_matrix(c)
        e, it, post, _ = oracle.decode_batch(c["algo"], H, a["syn"], c["p_phys"] / 3, c["max_iter"],
                                             a["layer_ptr"], a["layer_rows"], nthreads=4)
        for k in range(len(it)):
            if a["iters"][k] <= 30:
                short += 1
                assert it[k] == a["iters"][k], (c["id"], k)
                np.testing.assert_array_equal(e[k], a["ehat"][k])
                np.testing.assert_allclose(post[k], a["post"][k], rtol=1e-5, atol=0)
            else:
                long_ += 1
                long_same += int(it[k] == a["iters"][k] and np.array_equal(e[k], a["ehat"][k]))
    assert short >= 64 and long_ >= 24, (short, long_)
    assert long_same >= 0.85 * long_, (long_same, long_)
