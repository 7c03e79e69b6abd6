"""Dense NumPy restatement of the reference min-sum decoder — TEST / CPU-BASELINE
INFRASTRUCTURE ONLY (never imported by the product path).

What it is for: BASELINE.md "CPU-baseline plan" leg 1. It keeps the
reference's cost structure — per shot, dense m x n float32/float64 message
matrices, a full check-node pass over the layer's rows and a full dense
variable-node pass after every layer (qLDPCsim/decoders.py:147-177) — so that
`bench.py` can time "the reference algorithm as NumPy runs it" on the GPU
box's host cores, where the reference itself cannot travel. It is pinned
bit-exactly (hard decisions, iteration counts, float64 posteriors) to the
golden vectors captured from the unmodified reference
(tests/test_numpy_dense.py).

Numerical contract restated:
  * L = np.log((1-p)/max(p, eps)) is an np.float64 (decoders.py:147); the v2c
    matrix starts as float32(L) on edges (:148-149) and becomes float64 after
    the first variable-node pass (:177, NEP-50 promotion).
  * check node (:155-169): sign 0 -> +1, product of edge signs, min1 = first
    minimum, min2 = minimum with the first argmin removed, inf -> 0; an edge
    whose |v| equals min1 gets min2, others min1; value
    fl32(fl64(beta*syn_sign*prod*min) * sign_e).  Non-edges receive
    beta*syn*prod*min2/2 when min1 == 0 (the reference's "leak": its divisor
    sign + (1 - H) is 2 there), else 0.
  * variable node (:172-173): float32 column sums over all m rows (np.sum
    axis 0), posterior = L + sums in float64; stop test H e mod 2 == s after
    every layer (:175-176).
"""
import numpy as np

__all__ = ["DenseMinSum", "ms_decode_dense", "decode_batch_dense"]


class DenseMinSum:
    """Per-code dense state (masks reused across shots)."""

    def __init__(self, H, beta=0.75):
        self.H = (np.asarray(H) % 2).astype(np.int8)
        self.edge = self.H == 1
        self.m, self.n = self.H.shape
        self.beta = beta

    def decode(self, syndrome, p, max_iter, layers=None, eps=1e-9):
        """One shot -> (e_hat int8[n], iterations, posteriors f64[n])."""
        H, edge, beta = self.H, self.edge, self.beta
        m, n = self.m, self.n
        syndrome = np.asarray(syndrome)
        if layers is None:
            layers = [np.arange(m)]
        L = np.log((1 - p) / max(p, eps))                      # np.float64 (:147)
        v2c = np.where(edge, np.float32(L), np.float32(0.0))   # float32 until the first VN
        c2v = np.zeros((m, n), np.float32)
        ssign = np.where(syndrome == 1, -1.0, 1.0)[:, None]
        post = None
        e_hat = None
        for it in range(max_iter):
            for rows in layers:
                rows = np.asarray(rows)
                Er = edge[rows]
                V = v2c[rows]
                A = np.abs(V)
                Am = np.where(Er, A, np.inf)
                k = np.argmin(Am, axis=1)                        # first argmin
                r = np.arange(len(rows))
                min1 = Am[r, k]
                Am[r, k] = np.inf
                min2 = Am.min(axis=1)
                min1 = np.where(np.isinf(min1), 0.0, min1)[:, None]
                min2 = np.where(np.isinf(min2), 0.0, min2)[:, None]
                neg = (V < 0) & Er                               # sign 0 -> +1
                prod = np.where(np.count_nonzero(neg, axis=1) & 1, -1.0, 1.0)[:, None]
                scale = beta * ssign[rows] * prod                # exact: +-beta
                take2 = A == min1
                mag = np.where(take2, min2, min1)
                esign = np.where(neg, -1.0, 1.0)
                val = np.where(Er, (scale * mag) * esign, 0.0)
                # reference leak: non-edges see |0| == min1 when min1 == 0
                leak = (~Er) & take2
                if leak.any():
                    val = np.where(leak, (scale * min2) / 2.0, val)
                c2v[rows] = val.astype(np.float32)
                colsum = np.sum(c2v, axis=0)                     # float32, row order (:172)
                post = L + colsum                                # float64 (:173)
                e_hat = (post < 0).astype(np.int8)
                if np.array_equal(syndrome, H.dot(e_hat) % 2):   # (:175-176)
                    return e_hat, it + 1, post
                v2c = np.where(edge, post - c2v, 0.0)            # float64 from here (:177)
        return e_hat, max_iter, post


def ms_decode_dense(H, syndrome, p, max_iter, layers=None, beta=0.75, eps=1e-9):
    return DenseMinSum(H, beta).decode(syndrome, p, max_iter, layers, eps)


def decode_batch_dense(H, syn, p, max_iter, layers=None, beta=0.75, eps=1e-9):
    """Shots one at a time, as the reference's simulate_p loop does."""
    dec = DenseMinSum(H, beta)
    syn = np.asarray(syn)
    B = syn.shape[0]
    ehat = np.zeros((B, dec.n), np.uint8)
    iters = np.zeros(B, np.int32)
    post = np.zeros((B, dec.n), np.float64)
    for b in range(B):
        e, it, po = dec.decode(syn[b], p, max_iter, layers, eps)
        ehat[b], iters[b], post[b] = e, it, po
    return ehat, iters, post
