"""ms_flood_kernel's table image (capi.cpp flood_plain_layout /
flood_qc16_layout), inspected on the CPU through qldpc_schedule_flood_image:
the tables describe exactly H's Tanner graph with the reference's message
order (decoders.py:172-173: the column sum runs over ascending checks), and
the lift-16 layout of the headline code is free of LDS bank conflicts."""
import numpy as np
import pytest

from qldpcsim_amd import _lib, codes


def _image(H):
    m = H.shape[0]
    return _lib.flood_image(H, np.array([0, m], np.int32), np.arange(m, dtype=np.int32))


def _graph_checks(H, im):
    """Every live slot's words are its check's edges; every (check, column)
    message has its own slot, at the position the VN pass reads for its rank."""
    m, n = H.shape
    label = im["label"].astype(np.int64)
    assert len(set(label.tolist())) == n
    runs = [(int(im["start"][r]), int(im["count"][r]), int(im["deg"][r]), int(im["p0"][r]), int(im["stride"][r]))
            for r in range(im["n_runs"])]
    lab2col = {int(label[j]): j for j in range(n)}
    seen_slots = set()
    chk = im["chk"]
    assert sorted(c for c in chk.tolist() if c >= 0) == list(range(m))
    deg = int(H[0].sum())
    for s, c in enumerate(chk.tolist()):
        if c < 0:
            continue
        words = im["ftab"][s][:deg]
        labs = (words & 0xffff) // 8
        slots = (words >> 16) // 4
        assert sorted(lab2col[int(x)] for x in labs) == sorted(np.flatnonzero(H[c]).tolist())
        for lab, slot in zip(labs.tolist(), slots.tolist()):
            j = lab2col[lab]
            t = int(np.flatnonzero(H[:, j]).tolist().index(c))      # rank among the column's checks
            st, cnt, K, p0, S = next(r for r in runs if r[0] <= lab < r[0] + r[1])
            assert K == int(H[:, j].sum())
            o = lab - st
            assert slot == (p0 + t * S + o if S else p0 + o * K + t)
            assert slot not in seen_slots
            seen_slots.add(slot)
    assert len(seen_slots) == int(H.sum())


def _bank_cycles(im, deg):
    """LDS array cycles of the check-node pass per wave-iteration: per edge
    round and 32-lane group, the busiest bank's distinct addresses (post f64:
    label mod 32; messages f32: slot mod 32)."""
    tot = 0
    f = im["ftab"]
    for i in range(8):
        lanes = range(64 * i, 64 * i + 64)
        if all(im["chk"][q] < 0 for q in lanes):
            continue
        for k in range(deg):
            for g in (0, 32):
                grp = [64 * i + g + q for q in range(32)]
                for key in (lambda w: (w & 0xffff) // 8, lambda w: (w >> 16) // 4):
                    banks = {}
                    for q in grp:
                        a = int(key(int(f[q][k])))
                        banks.setdefault(a % 32, set()).add(a)
                    tot += max(len(v) for v in banks.values())
    return tot


@pytest.mark.parametrize("half", [0, 1])
def test_headline_code_gets_conflict_free_layout(half):
    H = codes.load_code("LP118_0")[half]
    im = _image(H)
    assert im is not None and im["qc"]
    _graph_checks(H, im)
    # 4 check slots x 8 rounds x 2 groups x (post + message): one cycle each
    assert _bank_cycles(im, 8) == 4 * 8 * 2 * 2
    # runs aligned to 32 labels, strides to 32 slots (whole-bank halves)
    for r in range(im["n_runs"]):
        assert im["start"][r] % 32 == 0 and im["p0"][r] % 32 == 0 and im["stride"][r] % 32 == 0


def test_plain_layout_when_not_lift16():
    """A uniform-degree code that is not lift-16 quasi-cyclic keeps the CSC
    layout (stride 0)."""
    rng = np.random.default_rng(3)
    Z, BR, BC = 15, 8, 20                    # lift 15: circulant blocks, 8 per block row
    H = np.zeros((BR * Z, BC * Z), np.uint8)
    eye = np.eye(Z, dtype=np.uint8)
    for R in range(BR):
        for C in rng.choice(BC, 8, replace=False):
            H[R * Z:(R + 1) * Z, C * Z:(C + 1) * Z] = np.roll(eye, int(rng.integers(Z)), axis=1)
    im = _image(H)
    assert im is not None and not im["qc"] and not im["stride"].any()
    _graph_checks(H, im)


def test_plain_env_forces_csc_layout(monkeypatch):
    """QLDPC_FLOOD_PLAIN=1 at schedule creation: the CSC layout for the
    headline code (the A/B switch the GPU parity test compares)."""
    monkeypatch.setenv("QLDPC_FLOOD_PLAIN", "1")
    H = codes.load_code("LP118_0")[0]
    code = _lib.Code(H)                        # uncached: a new schedule is built under the env
    m = H.shape[0]
    sched = _lib.Schedule(code, np.array([0, m], np.int32), np.arange(m, dtype=np.int32))
    import ctypes
    img, nb, ot, ol, qc = ctypes.c_void_p(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _lib.check(_lib.lib.qldpc_schedule_flood_image(sched.handle, ctypes.byref(img), ctypes.byref(nb),
                                                   ctypes.byref(ot), ctypes.byref(ol), ctypes.byref(qc)))
    assert img.value and qc.value == 0


@pytest.mark.gpu
def test_gpu_qc_layout_equals_plain_layout(monkeypatch):
    """The two layouts decode the same batch identically (iterations, hard
    decisions, flags, float64 posteriors), converging and non-converging
    syndromes of both halves of the headline code."""
    import torch
    from qldpcsim_amd import decoders
    for half in (0, 1):
        H = codes.load_code("LP118_0")[half]
        rng = np.random.default_rng(11 + half)
        e = (rng.random((6000, H.shape[1])) < 0.05).astype(np.int64)
        syn = np.concatenate([(e @ H.T.astype(np.int64)) % 2, rng.integers(0, 2, (500, H.shape[0]))]).astype(np.uint8)
        s = torch.as_tensor(syn, device="cuda")
        out = []
        for plain in (False, True):
            if plain:
                monkeypatch.setenv("QLDPC_FLOOD_PLAIN", "1")
            else:
                monkeypatch.delenv("QLDPC_FLOOD_PLAIN", raising=False)
            monkeypatch.setattr(_lib, "_code_cache", {})   # a fresh code + schedule under the env
            monkeypatch.setattr(_lib, "_code_fast", {})
            m = H.shape[0]
            im = _lib.flood_image(H, np.array([0, m], np.int32), np.arange(m, dtype=np.int32), 0)
            assert im["qc"] != plain
            out.append(decoders.decode_batch(H, s, 0.05 / 3, 50, algo="MS", want_post=True))
        torch.cuda.synchronize()
        a, b = out
        assert torch.equal(a.iters, b.iters) and torch.equal(a.ehat, b.ehat) and torch.equal(a.flags, b.flags)
        assert torch.equal(a.post.view(torch.int64), b.post.view(torch.int64))
