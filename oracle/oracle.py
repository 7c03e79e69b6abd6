"""ctypes front end of the C oracle (qldpc_oracle.c) — TEST INFRASTRUCTURE ONLY.

Parity pinned against golden vectors from the unmodified reference decoders
(tests/golden/gen_golden.py -> tests/test_oracle_golden.py).
The OSD restatement (`osd_dec`) is pure NumPy/Python, small cases only.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libqldpc_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        L.oracle_decode_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P,
                                          ctypes.c_int, P, P, P, ctypes.c_long, ctypes.c_double,
                                          ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                          P, P, P, P, ctypes.c_int]
        L.oracle_decode_batch.restype = ctypes.c_int
        U64 = ctypes.c_uint64
        L.oracle_channel_sample.argtypes = [ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int, P, P,
                                            U64, U64, U64, U64, U64, ctypes.c_long, P, P, P, P]
        L.oracle_channel_sample.restype = ctypes.c_int
        _lib = L
    return _lib


def csr(H):
    H = np.asarray(H)
    rows, cols = np.nonzero(H)            # row-major == np.where(H) edge order (decoders.py:224)
    row_ptr = np.zeros(H.shape[0] + 1, np.int32)
    np.add.at(row_ptr, rows + 1, 1)
    return np.cumsum(row_ptr, dtype=np.int64).astype(np.int32), cols.astype(np.int32)


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def decode_batch(algo, H, syn, p, max_iter, layer_ptr=None, layer_rows=None, beta=0.75,
                 eps=1e-9, want_post=True, nthreads=None):
    """Decode a batch of syndromes (uint8 [B, m]). algo: "MS" | "BP".

    Returns (ehat uint8[B,n], iters int32[B], post f64[B,n] | None, flags int32[B]).
    """
    H = np.asarray(H)
    m, n = H.shape
    rp, ci = csr(H)
    if layer_ptr is None:
        layer_ptr = np.array([0, m], np.int32)
        layer_rows = np.arange(m, dtype=np.int32)
    layer_ptr = np.ascontiguousarray(layer_ptr, np.int32)
    layer_rows = np.ascontiguousarray(layer_rows, np.int32)
    syn = np.ascontiguousarray(syn, np.uint8).reshape(-1, m)
    B = syn.shape[0]
    ehat = np.zeros((B, n), np.uint8)
    iters = np.zeros(B, np.int32)
    post = np.zeros((B, n), np.float64) if want_post else None
    flags = np.zeros(B, np.int32)
    rc = lib().oracle_decode_batch(0 if algo == "MS" else 1, m, n, _p(rp), _p(ci),
                                   len(layer_ptr) - 1, _p(layer_ptr), _p(layer_rows), _p(syn), B,
                                   float(p), int(max_iter), float(beta), float(eps), _p(ehat),
                                   _p(iters), _p(post), _p(flags),
                                   int(nthreads or os.cpu_count() or 1))
    if rc != 0:
        raise RuntimeError("oracle_decode_batch failed")
    return ehat, iters, post, flags


# --------------------------------------------------------------------------
# OSD restatement (decoders.py:299-370, gf2math.py:91-187). Small cases only.
# --------------------------------------------------------------------------
def _bits_to_int(v):
    """uint8/bool vector -> Python int with bit i = v[i]."""
    v = np.asarray(v, dtype=np.uint8) & 1
    return int.from_bytes(np.packbits(v, bitorder="little").tobytes(), "little") if v.size else 0


def gf2_rank(A):
    """gf2math.rank (gf2math.py:91-135): rank over GF(2), by an XOR basis of
    the bit-packed rows (same value as the reference's row reduction)."""
    A = np.asarray(A, dtype=np.uint8) & 1
    basis = {}
    r = 0
    for row in A:
        v = _bits_to_int(row)
        while v:
            h = v.bit_length() - 1
            if h not in basis:
                basis[h] = v
                r += 1
                break
            v ^= basis[h]
    return r


_RANK_CACHE = {}


def _rank_of(H):
    key = (H.shape, np.packbits(np.asarray(H, np.uint8) & 1).tobytes())
    if key not in _RANK_CACHE:
        _RANK_CACHE[key] = gf2_rank(H)
    return _RANK_CACHE[key]


def gf2_ref_T(A):
    """Transform T of gf2math.REF(A, reduced=True) (gf2math.py:139-187): the
    same pivot search and row operations, on bit-packed rows [A | T]."""
    A = (np.asarray(A) & 1).astype(np.uint8)
    nR, nC = A.shape
    W = nC + nR
    bits = np.zeros((nR, W), np.uint8)
    bits[:, :nC] = A
    bits[np.arange(nR), nC + np.arange(nR)] = 1
    words = (W + 63) // 64
    pk = np.packbits(bits, axis=1, bitorder="little")
    pk = np.concatenate([pk, np.zeros((nR, words * 8 - pk.shape[1]), np.uint8)], axis=1)
    R = pk.view(np.uint64).copy()                      # [nR, words]
    x = 0
    for c in range(nC):
        w, b = c >> 6, np.uint64(c & 63)
        col = ((R[:, w] >> b) & np.uint64(1)).astype(bool)
        cand = np.flatnonzero(col[x:])
        if cand.size == 0:
            continue
        r = x + int(cand[0])
        if r != x:
            R[[x, r]] = R[[r, x]]
            col[[x, r]] = col[[r, x]]
        # rows below the pivot, then rows above it, that hold a 1 in column c
        others = np.flatnonzero(col)
        others = others[others != x]
        R[others] ^= R[x]
        x += 1
        if x >= nR:
            break
    out = np.unpackbits(R.view(np.uint8), axis=1, bitorder="little")[:, nC:nC + nR]
    return out.astype(np.int8)


def osd_dec(H, e_hat, syndrome, post, order=0):
    """OSDdec restated (decoders.py:299-370), including its aliasing semantics."""
    H = (np.asarray(H) & 1).astype(np.int64)
    e_hat = np.asarray(e_hat).copy()
    post = np.asarray(post, dtype=np.float64)
    sat = np.where(np.abs(post) < 100.0, post, 100.0 * np.sign(post))
    prob = 1.0 / (1.0 + np.exp(sat))
    rel = np.where(prob > 0.5, prob, 1 - prob)
    perm = np.argsort(rel)
    Hp = H[:, perm]
    # Greedy complementary info set (decoders.py:329-342). The reference calls
    # gf2math.rank on Hp[:, J] after every append; "rank rose" is restated as
    # "the column is independent of the kept ones" with an incremental XOR
    # basis over bit-packed columns (same J, O(m) per column instead of a full
    # elimination). rank(Hp) = rank(H): a column permutation keeps the rank.
    colbytes = np.packbits(Hp.astype(np.uint8), axis=0, bitorder="little")
    cols = [int.from_bytes(colbytes[:, j].tobytes(), "little") for j in range(Hp.shape[1])]
    basis = {}

    def insert(v):
        while v:
            h = v.bit_length() - 1
            if h not in basis:
                basis[h] = v
                return True
            v ^= basis[h]
        return False

    max_rank = _rank_of(H)
    J = [0]
    past = 1 if insert(cols[0]) else 0
    nxt = 1
    while True:
        if nxt >= len(cols):
            raise IndexError(f"index {nxt} is out of bounds for axis 1 with size {len(cols)}")
        J.append(nxt)
        nxt += 1
        if not insert(cols[J[-1]]):
            J.pop()
            continue
        new = past + 1
        if new >= max_rank:
            break
        past = new
    info = list(set(range(H.shape[1])) - set(J))
    ep = e_hat[perm]
    T = gf2_ref_T(Hp[:, J])
    for w in range(2 ** order):
        flips = np.array([(w >> b) & 1 for b in range(len(info))])
        ep[info] ^= flips
        sJ = (np.asarray(syndrome) + Hp[:, info] @ ep[info]) % 2
        ep[J] = ((T.astype(np.int64) @ sJ) % 2)[:len(J)]
    e_hat[perm] = ep
    return e_hat


def channel_thresholds(p):
    """T_k = floor(k * (p/3) * 2^32), k = 1, 2, 3 (qldpc_channel_thresholds)."""
    q = p / 3.0
    return tuple(int(min(2.0 ** 32, np.floor((k + 1) * q * 2.0 ** 32))) for k in range(3))


def channel_sample(Hx, Hz, p, seed, shot0, batch):
    """Restatement of the device sampler stream (qldpc_channel_sample).

    Returns (sy_z, sy_x, errX, errZ) uint8 arrays, unpacked."""
    Hx = np.asarray(Hx)
    Hz = np.asarray(Hz)
    n = Hx.shape[1]
    rpx, cix = csr(Hx)
    rpz, ciz = csr(Hz)
    t1, t2, t3 = channel_thresholds(p)
    ex = np.zeros((batch, n), np.uint8)
    ez = np.zeros((batch, n), np.uint8)
    syz = np.zeros((batch, Hz.shape[0]), np.uint8)
    syx = np.zeros((batch, Hx.shape[0]), np.uint8)
    lib().oracle_channel_sample(n, Hx.shape[0], _p(rpx), _p(cix), Hz.shape[0], _p(rpz), _p(ciz),
                                t1, t2, t3, int(seed) & (2 ** 64 - 1), int(shot0), int(batch),
                                _p(ex), _p(ez), _p(syz), _p(syx))
    return syz, syx, ex, ez
