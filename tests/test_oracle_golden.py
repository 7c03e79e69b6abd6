"""Pin the CPU oracle against golden vectors from the unmodified reference.

MS and BP: hard decisions, iteration counts and float64 posteriors
bit-exact. BP is exact because include/qldpc_libm.h
restates NumPy's own tanh and SVML's atanh (and both decoders' np.log prior)
as NumPy runs them on the capture host.
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
    np.testing.assert_array_equal(post.view(np.uint64), a["post"].view(np.uint64))


def test_oracle_bp100_against_reference():
    """100-iteration BP golden set (configs[2] LP118_0 F/L, configs[4] LP118_2 L
    p-sweep, 8 shots per p and half, plus never-converging syndromes): BP at
    100 iterations is chaotic — it amplifies any last-bit difference in tanh /
    atanh into different hard decisions — so this pins the libm restatement:
    every shot, short or long, equal bit for bit (iterations, hard decisions,
    float64 posteriors)."""
    short = long_ = 0
    for c, a in BP100:
        H = half_matrix(c)
        e, it, post, _ = oracle.decode_batch(c["algo"], H, a["syn"], c["p_phys"] / 3, c["max_iter"],
                                             a["layer_ptr"], a["layer_rows"], nthreads=4)
        np.testing.assert_array_equal(it, a["iters"])
        np.testing.assert_array_equal(e, a["ehat"])
        np.testing.assert_array_equal(post.view(np.uint64), a["post"].view(np.uint64))
        short += int((a["iters"] <= 30).sum())
        long_ += int((a["iters"] > 30).sum())
    assert short >= 64 and long_ >= 24, (short, long_)


def test_oracle_osd_at_configs3_setting():
    """The oracle's OSD restatement (oracle.osd_dec) on the reference's final
    posteriors of configs[3]'s decodes (LP118_2 MS-L 50 it p = 0.1)
    reproduces the reference's OSD-0 and OSD-1 estimates."""
    n = 0
    for c, a in golden_cases("_osd50"):
        H = half_matrix(c)
        for k in np.flatnonzero(a["conv"] == 0):
            for order in (0, 1):
                got = oracle.osd_dec(H, a["ehat"][k].astype(np.int64), a["syn"][k].astype(np.int64),
                                     a["post"][k], order)
                np.testing.assert_array_equal(got.astype(np.uint8), a[f"ehat_osd{order}"][k])
            n += 1
    assert n >= 64, n
