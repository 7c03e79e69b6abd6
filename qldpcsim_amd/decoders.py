"""Drop-in decoders: the reference's decoders.py surface on the MI355X kernels.

    MS_decoder(H, syndrome, p, max_iter=99, layers=None, beta=0.75, OSDorder=-1, eps=1e-9)
        reference qLDPCsim/decoders.py:110-182  -> (e_hat int8[n], n_iter)
    BP_decoder(H, syndrome, p, max_iter=99, layers=None, OSDorder=-1, eps=1e-9)
        reference qLDPCsim/decoders.py:189-290  -> (e_hat int64[n], n_iter)
    OSDdec(H, e_hat, syndrome, posteriorLLRs, order=0)
        reference qLDPCsim/decoders.py:299-370  -> e_hat (updated in place)

plus the batched entry point the simulator uses, `decode_batch`, which decodes
many syndromes of one matrix in one kernel launch.

All decoding runs through the HIP kernels (libqldpc_hip.so via the C ABI);
there is no CPU fallback. OSD of the non-converged shots runs on the device
(osd_kernels.hip: NumPy's reliability order of decoders.py:320-325 — SVML's
exp and x86-simd-sort's argsort restated, ties included — and a block GF(2)
elimination); the rare shots the device order leaves to NumPy (a NaN
posterior, x86-simd-sort's std::sort fallback) get NumPy's own order on the
host and the device elimination again. `OSDdec` / `apply_osd` are the
single-shot and host entry points (host C++ elimination).

The restated order is NumPy 2.2.6's on x86-64 AVX512_SKX (the reference's
capture host). At first use, `numpy_order_pinned()` compares it with the running
NumPy on a fixed set of tie-heavy rows; if they differ (another NumPy build
or ISA dispatch), every OSD order is NumPy's own, computed on the host, and a
RuntimeWarning says why. `numpy_libm_pinned()` does the same for the tanh /
arctanh / log / exp restated for BP and the priors (BP is bit-exact only where
it holds; checked at the first BP decode); `parity_pins()` reports both.

Deviations from the reference (documented in DESIGN.md §7):
  * layers=None means flooding (the reference raises AttributeError on
    `np.range`, decoders.py:144 / :221).
  * H entries are reduced mod 2 (as load_matrix does, simulator.py:35);
    syndrome entries must be 0/1 (ValueError otherwise).
  * The min-sum "leak" case (a v2c message exactly 0.0, App. A.1.6) is
    flagged (FLAG_MIN_ZERO) but not emulated.
"""
import contextlib
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib, hostcores
from .schedule import pack_layers

__all__ = ["MS_decoder", "BP_decoder", "OSDdec", "decode_batch", "DecodeResult", "osd_perm", "pack_bits",
           "unpack_bits",
           "osd_perms", "apply_osd", "apply_osd_device", "apply_osd_device_many", "osd_device_stage",
           "osd_device_finish", "osd_host_orders", "osd_status_check", "numpy_order_pinned",
           "numpy_libm_pinned", "parity_pins"]


@dataclass
class DecodeResult:
    ehat: object          # uint8 [B, n]   (numpy, or torch on the device path)
    iters: object         # int32 [B]
    post: object          # float64 [B, n] or None
    flags: object         # int32 [B]

    @property
    def converged(self):
        return (self.flags & _lib.FLAG_CONVERGED) != 0


def _is_torch(x):
    return type(x).__module__.startswith("torch")


def pack_bits(bits):
    """uint8 [B, k] 0/1 tensor -> int64 [B, ceil(k/64)] words, bit j % 64 of
    word j / 64 (the bit-packed syndrome / estimate format, QLDPC_FMT_BITS)."""
    import torch
    B, k = bits.shape
    W = (k + 63) // 64
    x = torch.zeros((B, 64 * W), dtype=torch.int64, device=bits.device)
    x[:, :k] = bits.to(torch.int64) & 1
    sh = torch.arange(64, device=bits.device, dtype=torch.int64)
    return (x.view(B, W, 64) << sh).sum(dim=2)


def unpack_bits(words, k):
    """int64 [B, W] words -> uint8 [B, k] (inverse of pack_bits)."""
    import torch
    sh = torch.arange(64, device=words.device, dtype=torch.int64)
    return ((words.unsqueeze(-1) >> sh) & 1).to(torch.uint8).reshape(words.shape[0], -1)[:, :k]


def decode_batch(H, syndromes, p, max_iter, layers=None, algo="MS", beta=0.75, eps=1e-9,
                 want_post=False, osd_order=-1, layer_ptr=None, layer_rows=None, stream=None,
                 out=None, ehat_bits=False):
    """Decode a batch of syndromes of one matrix on the GPU.

    syndromes: uint8 [B, m] NumPy array (host; staged, synchronous) or a
    torch tensor on a HIP device (asynchronous on `stream` or torch's current
    stream; outputs are device tensors, OSD is not applied): uint8 [B, m] one
    byte per check, or int64 [B, ceil(m/64)] bit-packed words (pack_bits).
    `ehat_bits` (device path): hard decisions as int64 [B, ceil(n/64)] words
    instead of uint8 [B, n].
    `p` is the decoder prior (simulate passes p/3, simulator.py:278-282).
    `out` (device path): a DecodeResult of matching device tensors to write
    into instead of allocating (steady-state loops allocate nothing).
    """
    if algo not in _lib.ALGO:
        raise ValueError("Unrecognized decoder type.")
    if algo == "BP" and "libm" not in _PINNED:
        numpy_libm_pinned()                   # once: warns if BP cannot be bit-exact on this NumPy
    H = np.asarray(H)
    m, n = H.shape
    if layer_ptr is None:
        layer_ptr, layer_rows = pack_layers(layers, m)
    if int(max_iter) < 1:
        raise ValueError("max_iter must be >= 1")
    if _is_torch(syndromes):
        import torch
        dev = syndromes.device
        code = _lib.code_for(H, dev.index)
        sched = code.schedule(layer_ptr, layer_rows)
        syn = syndromes.contiguous()
        wm, wn = (m + 63) // 64, (n + 63) // 64
        if syn.dim() == 2 and syn.dtype == torch.uint8 and syn.shape[1] == m:
            syn_fmt = _lib.FMT_BYTES
        elif syn.dim() == 2 and syn.dtype == torch.int64 and syn.shape[1] == wm:
            syn_fmt = _lib.FMT_BITS
        else:
            raise ValueError(f"syndromes must be uint8 [B, {m}] or int64 words [B, {wm}]")
        B = syn.shape[0]
        e_shape, e_dtype = ((B, wn), torch.int64) if ehat_bits else ((B, n), torch.uint8)
        if out is not None:
            ehat, iters, flags, post = out.ehat, out.iters, out.flags, out.post if want_post else None
            ok = (ehat.shape == e_shape and ehat.dtype == e_dtype and iters.shape == (B,) and
                  iters.dtype == torch.int32 and flags.shape == (B,) and flags.dtype == torch.int32 and
                  all(t.device == dev and t.is_contiguous() for t in (ehat, iters, flags)) and
                  (not want_post or (post is not None and post.shape == (B, n) and
                                     post.dtype == torch.float64 and post.device == dev and
                                     post.is_contiguous())))
            if not ok:
                raise ValueError("out buffers do not match the batch (uint8 [B, n] or int64 [B, ceil(n/64)], "
                                 "int32 [B], int32 [B], float64 [B, n] if want_post) on the syndromes' device")
        else:
            ehat = torch.empty(e_shape, dtype=e_dtype, device=dev)
            iters = torch.empty(B, dtype=torch.int32, device=dev)
            flags = torch.empty(B, dtype=torch.int32, device=dev)
            post = torch.empty((B, n), dtype=torch.float64, device=dev) if want_post else None
        st = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        _lib.check(_lib.lib.qldpc_decode_device_ex(
            code.handle, sched.handle, _lib.ALGO[algo], syn.data_ptr(), syn_fmt, B, float(p), int(max_iter),
            float(beta), float(eps), ehat.data_ptr(), _lib.FMT_BITS if ehat_bits else _lib.FMT_BYTES,
            iters.data_ptr(), post.data_ptr() if post is not None else None, flags.data_ptr(), st))
        return DecodeResult(ehat, iters, post, flags)

    syn = np.ascontiguousarray(syndromes)
    if syn.ndim != 2 or syn.shape[1] != m:
        raise ValueError(f"syndromes must be [B, {m}]")
    if syn.size and (syn.min() < 0 or syn.max() > 1):
        raise ValueError("syndrome entries must be 0 or 1")
    syn = syn.astype(np.uint8, copy=False)
    B = syn.shape[0]
    code = _lib.code_for(H)
    sched = code.schedule(layer_ptr, layer_rows)
    ehat = np.zeros((B, n), np.uint8)
    iters = np.zeros(B, np.int32)
    flags = np.zeros(B, np.int32)
    need_post = want_post or osd_order >= 0
    post = np.zeros((B, n), np.float64) if need_post else None
    _lib.check(_lib.lib.qldpc_decode_host(
        code.handle, sched.handle, _lib.ALGO[algo], _lib.ptr(syn), B, float(p), int(max_iter),
        float(beta), float(eps), _lib.ptr(ehat), _lib.ptr(iters), _lib.ptr(post), _lib.ptr(flags)))
    res = DecodeResult(ehat, iters, post if want_post else None, flags)
    if osd_order >= 0:
        apply_osd(H, syn, ehat, post, flags, osd_order)
    return res


def osd_perm(posteriorLLRs):
    """Reliability order of decoders.py:320-325, computed with NumPy itself."""
    posteriorLLRs = np.asarray(posteriorLLRs)
    posteriorLLRsat = np.where(np.abs(posteriorLLRs) < 100.0, posteriorLLRs,
                               100.0 * np.sign(posteriorLLRs))
    posteriorProb = 1. / (1. + np.exp(posteriorLLRsat))
    reliability = np.where(posteriorProb > 0.5, posteriorProb, 1 - posteriorProb)
    return np.argsort(reliability)


def _pin_rows():
    """Fixed posterior rows for numpy_order_pinned: saturated (long runs of
    keys equal to 1.0), min-sum-quantised (many exact ties), +-x pairs, the
    clip edges, and sizes on both sides of the 256-key network."""
    rng = np.random.default_rng(20251226)
    rows = []
    L = np.log((1 - 0.1 / 3) / (0.1 / 3))
    for n in (7, 175, 256, 257, 544, 1020, 2047):
        P = rng.normal(0, 6, n)
        P[rng.random(n) < 0.7] *= 1e3
        rows.append(P)
        rows.append(L + rng.integers(-6, 7, n).astype(np.float32) * np.float32(0.975))
        Q = rng.normal(0, 2, n)
        Q[1::4] = -Q[::4][:Q[1::4].size]
        Q[:6] = [0.0, -0.0, 100.0, -100.0, 36.7, -36.7][:min(6, n)]
        rows.append(Q)
    return rows


_PINNED = {}                 # "order" / "libm" -> (bool, reason)


def _pin_warn(what, reason):
    import warnings
    warnings.warn(f"qldpcsim_amd: {what} not pinned to the running NumPy {np.__version__} ({reason}); "
                  + ("every OSD reliability order is computed by NumPy on the host (slower, same results)"
                     if what == "reliability order" else
                     "BP decodes follow the 1e-5 posterior contract instead of bit-exact parity"),
                  RuntimeWarning, stacklevel=3)


def numpy_order_pinned():
    """Whether the running NumPy's reliability order (np.exp, np.argsort)
    equals the restatement the device and the host library run
    (qldpc_osd_order_host): checked once, on _pin_rows(), bit for bit. When it
    does not, a RuntimeWarning says why (missing library symbol, or the first
    pin row whose order differs) and every OSD order is computed by NumPy on
    the host; parity_pins() reports the reason."""
    if "order" not in _PINNED:
        ok, why = True, "equal on every pin row"
        try:
            for r, P in enumerate(_pin_rows()):
                P = np.ascontiguousarray(P, np.float64)
                n = P.size
                perm = np.empty(n, np.int32)
                st = np.empty(1, np.int32)
                _lib.check(_lib.lib.qldpc_osd_order_host(_lib.ptr(P), 1, n, _lib.ptr(perm), _lib.ptr(st), 1))
                if st[0] != 0 or not np.array_equal(perm, osd_perm(P)):
                    ok, why = False, f"pin row {r} (n = {n}) orders differently"
                    break
        except (OSError, AttributeError, RuntimeError) as e:
            ok, why = False, f"{type(e).__name__}: {e}"
        _PINNED["order"] = (ok, why)
        if not ok:
            _pin_warn("reliability order", why)
    return _PINNED["order"][0]


def _libm_pin_args():
    """Fixed arguments for numpy_libm_pinned, over the ranges BP and the
    priors feed each function (decoders.py:147, :232, :254-259, :322)."""
    rng = np.random.default_rng(20251226)
    t = np.concatenate([rng.uniform(-40, 40, 6000), rng.uniform(-1, 1, 3000), rng.normal(0, 1e-4, 500),
                        np.linspace(19.0, 20.0, 257), -np.linspace(19.0, 20.0, 257),
                        [0.0, -0.0, 1e-300, -1e-300, 0.5, 24.0, 710.0, -710.0]])
    a = np.concatenate([rng.uniform(-1, 1, 6000), 1 - rng.uniform(0, 1e-6, 500), -1 + rng.uniform(0, 1e-6, 500),
                        [1 - 1e-9, -(1 - 1e-9), 0.0, -0.0, 1e-300, 0.5, -0.5]])
    pr = rng.uniform(1e-5, 0.4, 3000)
    lg = np.concatenate([(1 - pr) / pr, rng.uniform(1e-3, 1e3, 3000), np.exp(rng.uniform(-700, 700, 500))])
    ex = np.concatenate([rng.uniform(-100, 100, 6000), rng.uniform(-706, 706, 1000), [0.0, -0.0, 100.0, -100.0]])
    return {"tanh": (0, t, np.tanh), "atanh": (1, a, np.arctanh), "log": (2, lg, np.log), "exp": (3, ex, np.exp)}


def numpy_libm_pinned():
    """Whether the running NumPy's tanh / arctanh / log / exp equal the
    restatement BP's kernels and the priors run (include/qldpc_libm.h, through
    qldpc_libm_eval_host): checked once, bit for bit, on _libm_pin_args(). BP is
    bit-exact against the reference only where this holds;
    otherwise a RuntimeWarning says which function differs and parity_pins()
    reports it."""
    if "libm" not in _PINNED:
        ok, why = True, "equal on every pin argument"
        try:
            for name, (fn, x, ref) in _libm_pin_args().items():
                x = np.ascontiguousarray(x, np.float64)
                y = np.empty_like(x)
                _lib.check(_lib.lib.qldpc_libm_eval_host(fn, _lib.ptr(x), x.size, _lib.ptr(y)))
                with np.errstate(all="ignore"):
                    want = ref(x)
                bad = np.flatnonzero(y.view(np.uint64) != want.view(np.uint64))
                if bad.size:
                    ok, why = False, f"np.{ref.__name__} differs on {bad.size} of {x.size} arguments (x = {x[bad[0]]!r})"
                    break
        except (OSError, AttributeError, RuntimeError) as e:
            ok, why = False, f"{type(e).__name__}: {e}"
        _PINNED["libm"] = (ok, why)
        if not ok:
            _pin_warn("the restated libm", why)
    return _PINNED["libm"][0]


def parity_pins():
    """{"order": bool, "libm": bool, "numpy": version, "reasons": {...}}: the
    run-time pins parity depends on (smoke() and bench.py report them)."""
    numpy_order_pinned()
    numpy_libm_pinned()
    return {"order": _PINNED["order"][0], "libm": _PINNED["libm"][0], "numpy": np.__version__,
            "reasons": {k: v[1] for k, v in _PINNED.items()}}


def osd_perms(post, nthreads=None):
    """Row-wise reliability orders (decoders.py:320-325) of a [k, n] posterior
    block. When the running NumPy is the pinned one (numpy_order_pinned), the
    host library's restatement computes them (C++ threads, no GIL), and
    NumPy only the rows it leaves (NaN, std::sort fallback); otherwise NumPy's
    own exp / argsort, chunked over host threads (identical to per-row calls;
    NumPy releases the GIL in these loops)."""
    post = np.asarray(post)
    if post.shape[0] == 0:
        return np.zeros((0, post.shape[1]), np.int32)
    if numpy_order_pinned() and post.dtype == np.float64:
        P = np.ascontiguousarray(post)
        k, n = P.shape
        out = np.empty((k, n), np.int32)
        st = np.empty(k, np.int32)
        _lib.check(_lib.lib.qldpc_osd_order_host(_lib.ptr(P), k, n, _lib.ptr(out), _lib.ptr(st),
                                                 int(nthreads or hostcores.rank_cores())))
        for r in np.flatnonzero(st):
            out[r] = osd_perm(P[r])
        return out

    def one(P):
        # the reference's reliability, element for element (tests pin the bits):
        #   np.where(|P| < 100, P, 100 sign P)  ==  np.clip(P, -100, 100)
        #   1 / (1 + exp(sat))                  (same ufuncs, in place)
        #   np.where(prob > 0.5, prob, 1-prob)  ==  np.maximum(prob, 1-prob)
        #     (1 - prob is exact for prob > 0.5, and >= 0.5 >= prob otherwise)
        # 4x fewer passes over the block than the literal form, then NumPy's own
        # argsort decides the order (and its ties) exactly as the reference's.
        out = np.empty((P.shape[0], P.shape[1]), np.int32)
        for r0 in range(0, P.shape[0], 64):          # cache-sized row blocks
            t = np.clip(P[r0:r0 + 64], -100.0, 100.0)
            np.exp(t, out=t)
            np.add(t, 1.0, out=t)
            np.divide(1.0, t, out=t)
            np.maximum(t, np.subtract(1.0, t), out=t)
            out[r0:r0 + 64] = np.argsort(t, axis=1)
        return out

    nthreads = nthreads or hostcores.rank_cores()
    if post.shape[0] < 256 or nthreads <= 1:
        return one(post)
    # a persistent pool (starting 16 threads per call had cost ~4 ms, more than
    # the sorts of a few hundred rows) and chunks of >= 64 rows
    chunks = max(1, min(4 * nthreads, post.shape[0] // 64))
    return np.concatenate(list(_thread_pool(nthreads).map(one, np.array_split(post, chunks))))


_POOL = {}
_SIDE = {}


def _side_stream(dev):
    import torch
    if dev.index not in _SIDE:
        _SIDE[dev.index] = torch.cuda.Stream(dev)
    return _SIDE[dev.index]


def _thread_pool(n):
    from concurrent.futures import ThreadPoolExecutor
    if n not in _POOL:
        _POOL[n] = ThreadPoolExecutor(n)
    return _POOL[n]


_PINNED = {}


def _pinned(key, shape, dtype):
    """Grow-only page-locked host staging buffers (D2H of posteriors, H2D of
    reliability orders run at DMA speed instead of through pageable copies)."""
    import torch
    need = int(np.prod(shape))
    buf = _PINNED.get(key)
    if buf is None or buf.numel() < need or buf.dtype != dtype:
        # page-locking is slow (ms per call): grow geometrically, start at 1 MiB
        old = 0 if buf is None or buf.dtype != dtype else buf.numel()
        cap = max(need, 2 * old, (1 << 20) // torch.empty((), dtype=dtype).element_size())
        buf = torch.empty(cap, dtype=dtype, pin_memory=True)
        _PINNED[key] = buf
    return buf[:need].view(*shape)


def apply_osd_device(H, syn, res, order, stream=None):
    """GPU OSD for the non-converged shots of a device decode `res`
    (DecodeResult of torch tensors, with posteriors). The reliability order is
    NumPy's, computed on the device (qldpc_osd_device_ordered); only the shots
    it leaves to NumPy (NaN posteriors, x86-simd-sort's std::sort fallback)
    have their posteriors copied to the host. Updates res.ehat in place. See
    apply_osd_device_many for several decodes at once."""
    return apply_osd_device_many([(H, syn, res)], order, stream)[0]


def apply_osd_device_many(items, order, stream=None):
    """apply_osd_device for several (H, syn, res) decodes (the X and Z halves
    of a batch): every device order and elimination is queued first."""
    staged = osd_device_stage(items, stream, order=order)
    osd_device_finish(items, staged, order, stream)
    with _on_stream(stream):                      # the status check reads on the same stream
        osd_status_check(items)
    return [r.ehat for _, _, r in items]


# Where the OSD reliability order comes from (decoders.py:320-325):
#   device_min  fewest non-converged shots of one decode for which the order
#               is computed on the device (below it: on the host, after a copy
#               of their posteriors); the device order is NumPy's exact order,
#               so the default is every decode;
#   host_order  the host computes every OSD shot's order (A/B reference, and
#               the setting whenever the running NumPy is not the pinned one:
#               numpy_order_pinned() False).
# Read once at import from QLDPC_OSD_DEVICE_MIN / QLDPC_OSD_HOST_ORDER (tools
# start one process per setting); set_osd_policy / osd_policy change it.
OSD_POLICY = {"device_min": int(os.environ.get("QLDPC_OSD_DEVICE_MIN", "1")),
              "host_order": os.environ.get("QLDPC_OSD_HOST_ORDER", "") == "1"}


def set_osd_policy(device_min=None, host_order=None):
    if device_min is not None:
        OSD_POLICY["device_min"] = int(device_min)
    if host_order is not None:
        OSD_POLICY["host_order"] = bool(host_order)


@contextlib.contextmanager
def osd_policy(**kw):
    """`with osd_policy(device_min=1): ...` — the previous policy comes back after."""
    old = dict(OSD_POLICY)
    try:
        set_osd_policy(**kw)
        yield
    finally:
        OSD_POLICY.update(old)


# OSD shots of this process since reset_osd_stats(): every non-converged shot
# OSD saw, and those whose reliability order the host computed (NumPy or the
# host restatement: policy, n > 2048, or the device's NaN / fallback shots)
OSD_STATS = {"osd_shots": 0, "host_order_shots": 0}


def reset_osd_stats():
    OSD_STATS.update(osd_shots=0, host_order_shots=0)


def _host_order_only():
    return OSD_POLICY["host_order"] or not numpy_order_pinned()


def _device_order_min():
    return OSD_POLICY["device_min"]


def _on_stream(stream):
    """Context that makes `stream` (a raw HIP stream handle, or None = torch's
    current stream) the current stream, so every kernel, copy and event of
    one OSD stage is ordered on it."""
    import contextlib
    import torch
    if stream is None:
        return contextlib.nullcontext()
    return torch.cuda.stream(torch.cuda.ExternalStream(stream))


def release_workspaces():
    """Free the grow-only device OSD spill workspaces and pinned staging
    buffers (they are reused across batches while a sweep runs), and the HBM
    workspaces of every cached schedule (hbm_tile_kernel's message state:
    up to half the free device memory per schedule, kept between launches)."""
    _DEVBUF.clear()
    _PINNED.clear()
    _lib.release_hbm_workspaces()


def osd_device_stage(items, stream=None, slot0=0, order=0):
    """First half of the device OSD: find each decode's non-converged shots
    (one device sync), then queue asynchronously on the device: the
    reliability order (decoders.py:320-325) and the elimination of every shot
    whose result the device order decides, with its status copied into a
    pinned host buffer. Shots that need NumPy's order (status 2) are finished
    by osd_device_finish. `slot0` selects the pinned buffer set (pipelined
    callers alternate). OSD_POLICY["host_order"] (A/B, or an unpinned NumPy)
    or n > 2048 sends every shot through the host order (osd_perms)."""
    staged = []
    with _on_stream(stream):
        for slot, (H, syn, res) in enumerate(items):
            staged.append(_osd_stage_one(H, syn, res, slot0 + slot, order))
    return staged


def _osd_stage_one(H, syn, res, slot, order):
    import torch
    if res.post is None:
        raise ValueError("apply_osd_device needs the decode's posteriors (want_post=True)")
    m, n = np.shape(H)
    B = res.post.shape[0]
    # the OSD kernels read one byte per check / variable: bit-packed decodes
    # (ehat_bits, int64 word syndromes) must be unpacked first
    if not (syn.dtype == torch.uint8 and tuple(syn.shape) == (B, m)):
        raise ValueError(f"OSD needs uint8 [B, {m}] syndromes (unpack_bits a word batch first)")
    if not (res.ehat.dtype == torch.uint8 and tuple(res.ehat.shape) == (B, n)):
        raise ValueError(f"OSD needs uint8 [B, {n}] estimates (decode without ehat_bits)")
    dev = res.ehat.device
    bad = ((res.flags & _lib.FLAG_CONVERGED) == 0).nonzero().flatten()
    k = int(bad.numel())
    if k == 0:
        return None
    OSD_STATS["osd_shots"] += k
    n = res.post.shape[1]
    code = _lib.code_for(H, dev.index)
    post_b = res.post.index_select(0, bad)
    syn_b = syn.index_select(0, bad)
    e_b = res.ehat.index_select(0, bad)
    status = torch.empty(k, dtype=torch.int32, device=dev)
    cs = torch.cuda.current_stream(dev)
    st = cs.cuda_stream
    status_h = _pinned(("status", slot), (k,), torch.int32)
    on_dev = n <= 2048 and k >= _device_order_min() and not _host_order_only()
    spill = None
    if on_dev:
        perm = torch.empty((k, n), dtype=torch.int32, device=dev)
        tie = torch.empty(k, dtype=torch.int32, device=dev)
        # the shots left to NumPy's order copy their posteriors into a
        # spill buffer (one DMA copy for the host later, no gather kernel);
        # at most 256 MiB per buffer — a batch that spills more takes the
        # gather path in osd_device_finish
        cap = min(k // 2 + 1024, max(1024, (256 << 20) // (8 * n)))
        sp_post = _device_buf(("spill_post", slot), (cap, n), torch.float64, dev)
        sp_idx = _device_buf(("spill_idx", slot), (cap,), torch.int32, dev)
        sp_cnt = _device_buf(("spill_cnt", slot), (1,), torch.int32, dev)
        sp_cnt.zero_()
        _lib.check(_lib.lib.qldpc_osd_device_ordered_ex(
            code.handle, k, syn_b.data_ptr(), post_b.data_ptr(), int(order), e_b.data_ptr(),
            status.data_ptr(), perm.data_ptr(), tie.data_ptr(), sp_post.data_ptr(), sp_idx.data_ptr(),
            sp_cnt.data_ptr(), cap, st))
        cnt_h = _pinned(("spill_cnt", slot), (1,), torch.int32)
        cnt_h.copy_(sp_cnt, non_blocking=True)
        spill = (sp_post, sp_idx, cnt_h, cap)
    else:
        status.fill_(2)                            # every shot takes NumPy's order
    status_h.copy_(status, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(cs)
    return (bad, post_b, syn_b, e_b, status, status_h, ev, slot, on_dev, spill)


def osd_staged_on_device(staged):
    """Whether osd_device_stage queued any decode's shots with the device
    reliability order (rather than leaving them all to NumPy's)."""
    return any(sg is not None and sg[8] for sg in staged)


_DEVBUF = {}


def _device_buf(key, shape, dtype, dev):
    """Grow-only device workspaces reused across batches (per pipeline slot)."""
    import torch
    need = int(np.prod(shape))
    buf = _DEVBUF.get(key)
    if buf is None or buf.numel() < need or buf.dtype != dtype or buf.device != dev:
        buf = torch.empty(max(need, 1), dtype=dtype, device=dev)
        _DEVBUF[key] = buf
    return buf[:need].view(shape)


def osd_device_finish(items, staged, order, stream=None, host=None):
    """Second half: for each staged decode, the shots the device order could
    not decide (status 2) get NumPy's reliability order on the host (their
    posteriors only, pinned copies) and the GPU elimination; then the
    corrected estimates are scattered back, all queued asynchronously.
    `host` = the result of osd_host_orders(staged) if the caller already ran
    it (e.g. on a worker thread while the GPU ran the next batch); otherwise
    it runs here. res.osd_status keeps 0 / 1 per shot (1: the reference's
    IndexError case, raised by osd_status_check)."""
    if host is None:
        host = osd_host_orders(staged)
    with _on_stream(stream):
        for (H, syn, res), sg, hr in zip(items, staged, host):
            if sg is not None:
                _osd_finish_device(H, syn, res, sg, hr, order)
    return staged


def osd_host_orders(staged):
    """The host part of osd_device_finish, for every staged decode: wait for
    its device OSD (its event only), fetch the status-2 shots' posteriors and
    compute NumPy's reliability orders (decoders.py:320-325) for all of them
    in one pass over the host threads. Blocking, touches no launch stream, so
    a pipelined caller runs it on a worker thread while the GPU decodes the
    next batch. Returns per decode None (no staging) or (redo, perms_pinned)."""
    import torch
    out, blocks = [], []
    for sg in staged:
        if sg is None:
            out.append(None)
            continue
        bad, post_b, syn_b, e_b, status, status_h, ev, slot, _, spill = sg
        dev = post_b.device
        ev.synchronize()
        redo = (status_h.numpy() == 2).nonzero()[0]
        if redo.size == 0:
            out.append((redo, None))
            continue
        k2 = int(redo.size)
        hostp = _pinned(("post", slot), (k2, post_b.shape[1]), torch.float64)
        # fetch these posteriors on a side stream, with copies that wait only
        # for this decode's OSD (its event): the launch stream's next batch
        # (decode, device OSD) keeps running
        side = _side_stream(dev)
        side.wait_event(ev)
        if spill is not None and k2 <= spill[3] and int(spill[2][0]) == k2:
            # the kernels spilled exactly these rows: one contiguous DMA copy
            # (no gather kernel waiting for free CUs behind other work)
            sp_post, sp_idx, _, _ = spill
            idx_h = _pinned(("spill_idx", slot), (k2,), torch.int32)
            with torch.cuda.stream(side):
                hostp.copy_(sp_post[:k2], non_blocking=True)
                idx_h.copy_(sp_idx[:k2], non_blocking=True)
            side.synchronize()
            redo = idx_h.numpy().astype(np.int64)
        else:
            with torch.cuda.stream(side):
                idx_s = torch.as_tensor(redo, device=dev)
                hostp.copy_(post_b.index_select(0, idx_s), non_blocking=True)
            side.synchronize()
        out.append((redo, _pinned(("perm", slot), (k2, post_b.shape[1]), torch.int32)))
        blocks.append((len(out) - 1, hostp.numpy()))
    if blocks:
        # every decode's rows in one threaded pass (better parallel efficiency
        # than one pass per decode)
        if len(blocks) == 1 or len({b.shape[1] for _, b in blocks}) > 1:
            for i, P in blocks:
                out[i][1].numpy()[...] = osd_perms(P)
        else:
            perms = osd_perms(np.concatenate([P for _, P in blocks]))
            r0 = 0
            for i, P in blocks:
                out[i][1].numpy()[...] = perms[r0:r0 + P.shape[0]]
                r0 += P.shape[0]
    return out


def _osd_finish_device(H, syn, res, sg, hr, order):
    import torch
    bad, post_b, syn_b, e_b, status, status_h, ev, slot, _, spill = sg
    dev = res.ehat.device
    code = _lib.code_for(H, dev.index)
    redo, perm_h = hr
    res.osd_host_order = int(redo.size)
    OSD_STATS["host_order_shots"] += int(redo.size)
    if redo.size:
        k2 = int(redo.size)
        idx = torch.as_tensor(redo, device=dev)
        perms = perm_h.to(dev, non_blocking=True)
        syn_r = syn_b.index_select(0, idx)
        e_r = e_b.index_select(0, idx)
        st2 = torch.empty(k2, dtype=torch.int32, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(_lib.lib.qldpc_osd_device(code.handle, k2, syn_r.data_ptr(), perms.data_ptr(), int(order),
                                             e_r.data_ptr(), st2.data_ptr(), st))
        e_b.index_copy_(0, idx, e_r)
        status.index_copy_(0, idx, st2)
    res.ehat.index_copy_(0, bad, e_b)
    res.osd_status = status      # checked by the caller (raises IndexError like the reference)


def osd_status_check(items, defer=None):
    """Raise the reference's IndexError if any OSD of these decodes ran its
    greedy basis loop past the last column (decoders.py:333-342). With a
    `defer` list, the per-decode flags are appended there as device tensors
    instead (no sync; the caller checks them with osd_status_raise)."""
    for _, _, res in items:
        st = getattr(res, "osd_status", None)
        if st is None:
            continue
        if defer is not None:
            defer.append((st != 0).any())
        elif bool((st != 0).any()):
            raise IndexError("OSD: column basis search ran past the last column")


def osd_status_raise(flags):
    """osd_status_check's deferred flags: one sync for all of them."""
    import torch
    if flags and bool(torch.stack(flags).any()):
        raise IndexError("OSD: column basis search ran past the last column")


def apply_osd(H, syn, ehat, post, flags, order, nthreads=None):
    """OSD post-step for every non-converged row (decoders.py:179-180, :287-288).

    ehat (uint8 [B, n]) is updated in place.
    """
    idx = np.flatnonzero((np.asarray(flags) & _lib.FLAG_CONVERGED) == 0)
    if idx.size == 0:
        return ehat
    OSD_STATS["osd_shots"] += int(idx.size)
    OSD_STATS["host_order_shots"] += int(idx.size)
    code = _lib.code_for(H)
    perms = np.ascontiguousarray(osd_perms(post[idx]), dtype=np.int32)
    sub_syn = np.ascontiguousarray(syn[idx], dtype=np.uint8)
    sub_e = np.ascontiguousarray(ehat[idx], dtype=np.uint8)
    _lib.check(_lib.lib.qldpc_osd_decode_batch(code.handle, idx.size, _lib.ptr(sub_syn),
                                               _lib.ptr(perms), int(order), _lib.ptr(sub_e),
                                               int(nthreads or hostcores.rank_cores())))
    ehat[idx] = sub_e
    return ehat


def _single(H, syndrome, p, max_iter, layers, algo, beta, eps):
    H = np.asarray(H)
    syndrome = np.asarray(syndrome)
    m, n = H.shape
    if syndrome.shape != (m,):
        raise ValueError(f"syndrome must have shape ({m},), got {syndrome.shape}")
    if int(max_iter) < 1:
        # the reference's iteration loop never binds e_hat (decoders.py:153/:182)
        raise UnboundLocalError("local variable 'e_hat' referenced before assignment")
    lp, lr = pack_layers(layers, m)
    r = decode_batch(H, syndrome.reshape(1, m), p, max_iter, algo=algo, beta=beta, eps=eps,
                     want_post=True, layer_ptr=lp, layer_rows=lr)
    return r.ehat[0], int(r.iters[0]), r.post[0], bool(r.converged[0])


def MS_decoder(H: np.ndarray, syndrome: np.ndarray, p: float, max_iter: int = 99,
               layers: Optional[list] = None, beta: float = 0.75, OSDorder: int = -1,
               eps: float = 1e-9):
    """Normalized min-sum (reference decoders.py:110-182) on the GPU."""
    H = np.asarray(H)
    syndrome = np.asarray(syndrome)
    if H.size == 0 or syndrome.size == 0:          # reference quirk: bare array (:138-139)
        return np.zeros(H.shape[1] if H.size else 0, dtype=np.int8)
    e, it, post, conv = _single(H, syndrome, p, max_iter, layers, "MS", beta, eps)
    e_hat = e.astype(np.int8)
    if not conv and OSDorder >= 0:                 # (:179-180)
        e_hat = OSDdec(H, e_hat, syndrome, post, OSDorder)
    return e_hat, it


def BP_decoder(H: np.ndarray, syndrome: np.ndarray, p: float, max_iter: int = 99,
               layers: Optional[list] = None, OSDorder: int = -1, eps: float = 1e-9):
    """Sum-product BP (reference decoders.py:189-290) on the GPU."""
    H = np.asarray(H)
    syndrome = np.asarray(syndrome)
    if H.size == 0 or syndrome.size == 0:          # (:215-216)
        return np.zeros(H.shape[1] if H.size else 0, dtype=np.int8)
    e, it, post, conv = _single(H, syndrome, p, max_iter, layers, "BP", 0.75, eps)
    e_hat = e.astype(int)                          # (L_post < 0).astype(int) (:280)
    if not conv and OSDorder >= 0:                 # (:287-288)
        e_hat = OSDdec(H, e_hat, syndrome, post, OSDorder)
    return e_hat, it


def OSDdec(H: np.ndarray, e_hat: np.ndarray, syndrome: np.ndarray, posteriorLLRs: np.ndarray,
           order: int = 0) -> np.ndarray:
    """OSD post-decoder (reference decoders.py:299-370), host C++ GF(2).

    Mutates and returns `e_hat`, like the reference's `e_hat[perm] = ...`.
    """
    H = np.asarray(H)
    m, n = H.shape
    perm = np.ascontiguousarray(osd_perm(posteriorLLRs), dtype=np.int32)
    syn = np.ascontiguousarray(np.asarray(syndrome) % 2, dtype=np.uint8)
    e = np.ascontiguousarray(np.asarray(e_hat) & 1, dtype=np.uint8)
    code = _lib.code_for(H)
    _lib.check(_lib.lib.qldpc_osd_decode(code.handle, _lib.ptr(syn), _lib.ptr(perm), int(order),
                                         _lib.ptr(e), None, None, -1))
    e_hat[...] = e.astype(e_hat.dtype)
    return e_hat
