"""Monte-Carlo driver with the reference simulator's API, batched on the GPU.

Same names, arguments, flags and counters as albertogp71/qLDPCsim
qLDPCsim/simulator.py:
    load_matrix(path)                                   simulator.py:20-35
    simulate_p(Hx, Hz, p, shots, decType, decIterations,
               decSchedule, OSDorder, rngSeed) -> dict  simulator.py:167-315
    simulate(HxFile, HzFile, p, shots, ...)             simulator.py:319-347
    main(argv)                                          simulator.py:351-373

What changes underneath: instead of a serial Python loop over shots
(simulator.py:244-304) the shots are processed in batches — one kernel
launch per half (X: Hz with the Hx-derived layers; Z: Hx with the
Hz-derived layers, the reference's cross-wiring, :278-282) — and the counters
are formed with array operations with the reference's exact definitions.
With torch.distributed initialised, shots shard across ranks and the six
counters are summed with one all_reduce (RCCL over xGMI on the GPU node);
`torchrun --nproc-per-node 8 -m qldpcsim_amd.simulator ...` sets that up
(one process per GPU).

Syndrome source: Stim is not available in this environment,
so shots come from a per-qubit Pauli sampler (X, Y, Z each p/3 — the
circuit's PAULI_CHANNEL_1(p/3,p/3,p/3), simulator.py:107) whose statistics
equal the circuit's: on the GPU a counter-based Philox
stream drawn by a HIP kernel next to the outcome counters (DeviceChannel,
channel_kernels.hip); on the host NumPy's generator (sample_channel). `rngSeed` seeds it (the reference
seeds np.random, which its unseeded Stim sampler never reads: runs there are
not reproducible; here they are).
"""
import argparse
import sys
import time
from typing import Optional

# smallest tapered tail batch = batch_size // TAIL_DIV (see the tail tapering
# below; 32 vs 8: +0.5 % on configs[3] p = 0.1, profiles/r04bb/)
TAIL_DIV = 32

import numpy as np

from . import _lib, decoders
from .schedule import layerize, select_layers, pack_layers  # noqa: F401  (re-exported)

__all__ = ["load_matrix", "simulate_p", "simulate", "main", "layerize", "sample_channel",
           "count_outcomes"]

COUNTER_KEYS = ("DecFailures_X", "DecFailures_Z", "decSuccessExact", "decSuccessDegen",
                "nIterAccX", "nIterAccZ")


def load_matrix(path: str) -> np.ndarray:
    """Load a binary matrix from .npy or whitespace text (simulator.py:20-35)."""
    if path.endswith(".npy"):
        mat = np.load(path, allow_pickle=False)
    else:
        mat = []
        with open(path, "rt") as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                mat.append([int(x) for x in line.split()])
        mat = np.array(mat, dtype=int)
    return (mat % 2).astype(np.int8)


def sample_channel(Hx, Hz, p, shots, rng):
    """Depolarizing-channel samples in the circuit's output layout.

    Returns (sy_z, sy_x, errX, errZ) as uint8 arrays ([shots, m_z], [shots, m_x],
    [shots, n], [shots, n]) — the slices simulator.py:249-252 takes of a Stim
    sample row [sy_z | sy_x | errX | errZ].
    """
    n = Hx.shape[1]
    u = rng.random((shots, n), dtype=np.float32)
    q = np.float32(p / 3)
    X = u < q
    Y = (u >= q) & (u < 2 * q)
    Z = (u >= 2 * q) & (u < np.float32(p))
    errX = (X | Y).astype(np.uint8)
    errZ = (Z | Y).astype(np.uint8)
    # H·e mod 2 via a float32 product (exact: row weights << 2^24)
    sy_z = (errX.astype(np.float32) @ Hz.T.astype(np.float32)).astype(np.int64) % 2
    sy_x = (errZ.astype(np.float32) @ Hx.T.astype(np.float32)).astype(np.int64) % 2
    return sy_z.astype(np.uint8), sy_x.astype(np.uint8), errX, errZ


def count_outcomes(Hx, Hz, sy_z, sy_x, errX, errZ, eX, eZ, itX, itZ):
    """The reference's per-shot outcome counting (simulator.py:291-303), vectorised.

    exact:  errX == eX_hat and errZ == eZ_hat                       (:294-295)
    degen:  otherwise, Hz @ (errX ^ eX_hat) == 0 and Hx @ (errZ ^ eZ_hat) == 0
            over the integers, no mod 2 (:296-298; the reference also calls
            breakpoint() there)
    failX/Z: syndrome of the estimate differs from the measured one (:300-303)
    """
    exact = np.all(errX == eX, axis=1) & np.all(errZ == eZ, axis=1)
    dX = (errX ^ eX).astype(np.float32)
    dZ = (errZ ^ eZ).astype(np.float32)
    degen = (~exact) & np.all(dX @ Hz.T.astype(np.float32) == 0, axis=1) & \
        np.all(dZ @ Hx.T.astype(np.float32) == 0, axis=1)
    sX = (eX.astype(np.float32) @ Hz.T.astype(np.float32)).astype(np.int64) % 2
    sZ = (eZ.astype(np.float32) @ Hx.T.astype(np.float32)).astype(np.int64) % 2
    failX = np.any(sX != sy_z, axis=1)
    failZ = np.any(sZ != sy_x, axis=1)
    return {
        "DecFailures_X": int(failX.sum()),
        "DecFailures_Z": int(failZ.sum()),
        "decSuccessExact": int(exact.sum()),
        "decSuccessDegen": int(degen.sum()),
        "nIterAccX": int(np.asarray(itX, dtype=np.int64).sum()),
        "nIterAccZ": int(np.asarray(itZ, dtype=np.int64).sum()),
    }


class DeviceChannel:
    """Device-side shot source and outcome counters (channel_kernels.hip via
    the C ABI): the depolarizing draw of `sample_channel` as a counter-based
    Philox stream (qldpc_channel_sample: shot s of seed k is the same whatever
    the batching) and the counter definitions of `count_outcomes`
    (qldpc_count_outcomes), so a batch never leaves HBM.

    sample() returns (sy_z uint8 [B, m_z], sy_x uint8 [B, m_x], errX, errZ)
    with errX / errZ bit-packed as int64 [B, ceil(n/64)] words (bit j % 64 of
    word j / 64); `unpack` turns them into uint8 [B, n]."""

    def __init__(self, Hx, Hz, device, seed, shot0=0):
        import torch
        self.torch = torch
        self.dev = torch.device(device)
        self.n = Hx.shape[1]
        self.W = (self.n + 63) // 64
        with torch.cuda.device(self.dev):
            self.cx = _lib.code_for(Hx, self.dev.index)
            self.cz = _lib.code_for(Hz, self.dev.index)
        self.mx, self.mz = self.cx.m, self.cz.m
        self.seed = int(seed) & ((1 << 64) - 1)
        self.shot = int(shot0)

    def _stream(self):
        return self.torch.cuda.current_stream(self.dev).cuda_stream

    def sample(self, p, B, bits=False):
        """`bits`: syndromes as int64 words [B, ceil(m/64)] (decode_batch
        reads either format) instead of uint8 [B, m]."""
        torch = self.torch
        errX = torch.empty((B, self.W), dtype=torch.int64, device=self.dev)
        errZ = torch.empty((B, self.W), dtype=torch.int64, device=self.dev)
        if bits:
            sy_z = torch.empty((B, (self.mz + 63) // 64), dtype=torch.int64, device=self.dev)
            sy_x = torch.empty((B, (self.mx + 63) // 64), dtype=torch.int64, device=self.dev)
        else:
            sy_z = torch.empty((B, self.mz), dtype=torch.uint8, device=self.dev)
            sy_x = torch.empty((B, self.mx), dtype=torch.uint8, device=self.dev)
        _lib.check(_lib.lib.qldpc_channel_sample_ex(
            self.cx.handle, self.cz.handle, float(p), self.seed, self.shot, int(B), errX.data_ptr(),
            errZ.data_ptr(), sy_z.data_ptr(), sy_x.data_ptr(), _lib.FMT_BITS if bits else _lib.FMT_BYTES,
            self._stream()))
        self.shot += int(B)
        return sy_z, sy_x, errX, errZ

    def unpack(self, words):
        """Packed int64 [B, W] error words -> uint8 [B, n] (device)."""
        torch = self.torch
        bits = torch.arange(64, device=words.device, dtype=torch.int64)
        return ((words.unsqueeze(-1) >> bits) & 1).to(torch.uint8).reshape(words.shape[0], -1)[:, :self.n]

    def count_device(self, sy_z, sy_x, errX, errZ, eX, eZ, itX, itZ, acc=None):
        """Adds the batch's six counters (COUNTER_KEYS order) to `acc`
        (int64 [6] device tensor, created if None) without a host sync."""
        torch = self.torch
        if acc is None:
            acc = torch.zeros(len(COUNTER_KEYS), dtype=torch.int64, device=self.dev)
        B = sy_z.shape[0]
        ts = (sy_z, sy_x, errX, errZ, eX, eZ, itX, itZ)
        syn_bits = sy_z.dtype == torch.int64
        e_bits = eX.dtype == torch.int64
        e_shape = (B, self.W) if e_bits else (B, self.n)
        if not all(t.is_contiguous() and t.device == self.dev for t in ts) or \
                eX.shape != e_shape or eZ.shape != e_shape or errX.shape != (B, self.W) or \
                eX.dtype not in (torch.uint8, torch.int64) or eZ.dtype != eX.dtype or \
                sy_x.dtype != sy_z.dtype or itX.dtype != torch.int32 or itZ.dtype != torch.int32:
            raise ValueError("count_device: buffers do not match the batch layout")
        F = lambda b: _lib.FMT_BITS if b else _lib.FMT_BYTES  # noqa: E731
        _lib.check(_lib.lib.qldpc_count_outcomes_ex(
            self.cx.handle, self.cz.handle, int(B), errX.data_ptr(), errZ.data_ptr(), sy_z.data_ptr(),
            sy_x.data_ptr(), F(syn_bits), eX.data_ptr(), eZ.data_ptr(), F(e_bits), itX.data_ptr(),
            itZ.data_ptr(), acc.data_ptr(), self._stream()))
        return acc

    def count(self, sy_z, sy_x, errX, errZ, eX, eZ, itX, itZ):
        v = self.count_device(sy_z, sy_x, errX, errZ, eX, eZ, itX, itZ).cpu().tolist()
        return dict(zip(COUNTER_KEYS, (int(x) for x in v)))


def _device_ok():
    try:
        import torch
        return torch.cuda.is_available()
    except ImportError:
        return False


def _channel_ok(Hx, Hz):
    """The device sampler / counters handle n <= 4096 qubits (64 error words
    per shot, qldpc_channel_sample); larger codes use the host sampler."""
    return Hx.shape[1] <= 4096 and Hx.shape[1] == Hz.shape[1]


def _dist():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist, dist.get_rank(), dist.get_world_size()
    except ImportError:
        pass
    return None, 0, 1


_WORKER = []


def _host_worker():
    """One background thread for the pipelined OSD's host work (waiting for a
    batch's device OSD, fetching the status-2 posteriors, NumPy's orders), so
    the main thread keeps queueing the next batch's GPU work."""
    from concurrent.futures import ThreadPoolExecutor
    if not _WORKER:
        _WORKER.append(ThreadPoolExecutor(1))
    return _WORKER[0]


def _host_orders_on(dev, staged):
    """decoders.osd_host_orders on the worker thread, with this rank's device
    current there too (the HIP current device is per thread)."""
    import torch
    torch.cuda.set_device(dev)
    return decoders.osd_host_orders(staged)


def simulate_p(Hx: np.ndarray, Hz: np.ndarray, p: float, shots: int = 1000, decType: str = "MS",
               decIterations: int = 99, decSchedule: str = "F", OSDorder: int = -1,
               rngSeed: Optional[int] = None, *, batch_size: Optional[int] = None,
               verbose: bool = True, samples=None, sampler: Optional[str] = None) -> dict:
    """One depolarizing probability: sample, decode both halves, count.

    Returns the reference's dict (simulator.py:308-315). `samples`, if given,
    is a tuple (sy_z, sy_x, errX, errZ) to decode instead of sampling (used by
    the parity tests). `sampler`: "device" (HIP sampler + counters on the GPU,
    the default when a device is present), or "host" (NumPy). Extra keyword
    arguments default to reference behaviour.
    """
    if rngSeed is not None:
        np.random.seed(rngSeed)                    # reference side effect (:187-188)
    dist, rank, world = _dist()
    m_z = Hz.shape[0] if Hz.size else 0
    m_x = Hx.shape[0] if Hx.size else 0
    n = Hx.shape[1]
    if Hz.size and Hz.shape[1] != n:
        raise ValueError("Hx and Hz must have the same number of columns (physical qubits).")
    layersX, layersZ = select_layers(Hx, Hz, decSchedule)   # raises ValueError (:236)
    if decType in ("NG", "BF"):
        raise NotImplementedError(
            f"decType {decType!r} (decoders.py NG_decoder/BF_decoder) is outside the MI355X "
            "decoder's scope (SURVEY.md §2 rows 4-5); use 'MS' or 'BP'")
    if decType not in ("MS", "BP"):
        raise ValueError("Unrecognized decoder type.")
    # the reference never passes OSDorder to BP_decoder (:281-282)
    osd = OSDorder if decType == "MS" else -1
    lpX, lrX = pack_layers(layersX, Hz.shape[0])    # X half decodes Hz with Hx's layers
    lpZ, lrZ = pack_layers(layersZ, Hx.shape[0])    # Z half decodes Hx with Hz's layers

    # this rank's contiguous share of the shots
    my_shots = shots // world + (1 if rank < shots % world else 0)
    my_start = rank * (shots // world) + min(rank, shots % world)
    seed = None if rngSeed is None else [int(rngSeed), int(rank)]
    rng = np.random.default_rng(seed)
    tot = {k: 0 for k in COUNTER_KEYS}
    t0 = time.time()
    done = 0
    if sampler not in (None, "device", "host"):
        raise ValueError("sampler must be 'device', 'host' or None")
    if samples is not None and sampler == "device":
        raise ValueError("samples= decodes the given shots on the host path; it cannot be combined "
                         "with sampler='device' (which draws its own Philox shots)")
    use_dev = sampler == "device" or (sampler is None and samples is None and _device_ok()
                                      and _channel_ok(Hx, Hz))
    if batch_size is None:
        # shots per batch. Without OSD nothing syncs per batch, and 2^20-shot
        # batches amortise the per-batch host work (LP118_0 MS-F p = 0.01:
        # 107 -> 130 M shots/s vs 2^18); with OSD, 2^18 keeps the host's
        # reliability order of one batch overlapped with the next one's decode.
        batch_size = ((1 << 20) if osd < 0 else (1 << 18)) if use_dev else (1 << 16)
    if use_dev:
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        ch = DeviceChannel(Hx, Hz, dev, np.random.SeedSequence(seed).generate_state(1, np.uint64)[0])
    if use_dev:
        # Two-stage pipeline over batches: the host computes batch b-1's OSD
        # reliability orders (NumPy, the shots the device order leaves) while
        # the GPU runs batch b's decode and device OSD;
        # counters accumulate on the device (one sync per batch, in the OSD
        # staging; none without OSD until the end).
        acc = torch.zeros(len(COUNTER_KEYS), dtype=torch.int64, device=dev)
        pending = None
        phase = 0
        osd_flags = []                             # IndexError flags, checked once at the end
        stage_first = False                        # the last batch had device-ordered OSD shots
        tail_min = max(1, batch_size // TAIL_DIV)
        osd_frac = 0.0                             # OSD shots / half-shots of the last staged batch
        while done < my_shots or pending is not None:
            cur = None
            if done < my_shots:
                rem = my_shots - done
                B = min(batch_size, rem)
                if osd >= 0 and osd_frac > 0.2 and tail_min < rem <= batch_size:
                    # the last batch's NumPy orders have no next batch to hide
                    # behind (the GPU idles until they finish): when OSD is a
                    # large share of the work, halve the tail batches, so the
                    # final wait is a small batch's (LP118_2 MS-L p = 0.1:
                    # +5 %; at low p the extra batches cost more than the
                    # short drain saves). Shots keep their indices (the
                    # sampler's counter): counters do not depend on batching.
                    B = max(tail_min, rem // 2)
                # bit-packed syndromes and estimates (one bit per check / qubit
                # in HBM) unless OSD needs byte rows of the failing shots
                packed = osd < 0
                sy_z, sy_x, errX, errZ = ch.sample(p, B, bits=packed)
                want_post = osd >= 0
                rX = decoders.decode_batch(Hz, sy_z, p / 3, decIterations, algo=decType, want_post=want_post,
                                           layer_ptr=lpX, layer_rows=lrX, ehat_bits=packed)
                rZ = decoders.decode_batch(Hx, sy_x, p / 3, decIterations, algo=decType, want_post=want_post,
                                           layer_ptr=lpZ, layer_rows=lrZ, ehat_bits=packed)
                cur = [sy_z, sy_x, errX, errZ, rX, rZ, None]
                done += B
            if cur is not None and osd >= 0 and stage_first:
                # many OSD shots: this batch's device OSD is queued first
                # (staging waits for its decode), so the GPU runs it while the
                # worker thread finishes the previous batch's NumPy orders
                cur[6] = decoders.osd_device_stage([(Hz, cur[0], cur[4]), (Hx, cur[1], cur[5])],
                                                   slot0=2 * phase, order=osd)
                cur.append(_host_worker().submit(_host_orders_on, dev, cur[6]))
                phase ^= 1
            if pending is not None:
                sy_z_, sy_x_, errX_, errZ_, rX_, rZ_, staged = pending[:7]
                items = [(Hz, sy_z_, rX_), (Hx, sy_x_, rZ_)]
                if osd >= 0:                           # (decoders.py:179-180), on the GPU
                    # the status-2 shots' NumPy orders were computed on the
                    # worker thread while the GPU decoded this batch
                    decoders.osd_device_finish(items, staged, osd, host=pending[7].result())
                    decoders.osd_status_check(items, defer=osd_flags)
                ch.count_device(sy_z_, sy_x_, errX_, errZ_, rX_.ehat, rZ_.ehat, rX_.iters, rZ_.iters, acc)
            if cur is not None and osd >= 0 and cur[6] is None:
                # few OSD shots: stage (and sync on) this batch's decode now
                cur[6] = decoders.osd_device_stage([(Hz, cur[0], cur[4]), (Hx, cur[1], cur[5])],
                                                   slot0=2 * phase, order=osd)
                cur.append(_host_worker().submit(_host_orders_on, dev, cur[6]))
                phase ^= 1
            if cur is not None and osd >= 0:
                stage_first = decoders.osd_staged_on_device(cur[6])
                osd_frac = sum(int(sg[0].numel()) for sg in cur[6] if sg is not None) / (2.0 * B)
            pending = cur
            if verbose and rank == 0 and cur is not None:
                print(f"\r(p={p:5.2e}) Decoding block n. {done:3}/{my_shots:4}... "
                      f"({done / (time.time() - t0):.3g} shots/s)", end="", flush=True)
        decoders.osd_status_raise(osd_flags)
        tot = dict(zip(COUNTER_KEYS, (int(x) for x in acc.cpu().tolist())))
    while not use_dev and done < my_shots:
        B = min(batch_size, my_shots - done)
        if samples is not None:
            sl = slice(my_start + done, my_start + done + B)
            sy_z, sy_x, errX, errZ = (np.asarray(a)[sl].astype(np.uint8) for a in samples)
        else:
            sy_z, sy_x, errX, errZ = sample_channel(Hx, Hz, p, B, rng)
        rX = decoders.decode_batch(Hz, sy_z, p / 3, decIterations, algo=decType, osd_order=osd,
                                   layer_ptr=lpX, layer_rows=lrX)
        rZ = decoders.decode_batch(Hx, sy_x, p / 3, decIterations, algo=decType, osd_order=osd,
                                   layer_ptr=lpZ, layer_rows=lrZ)
        c = count_outcomes(Hx, Hz, sy_z, sy_x, errX, errZ, rX.ehat, rZ.ehat, rX.iters, rZ.iters)
        for k in tot:
            tot[k] += c[k]
        done += B
        if verbose and rank == 0:
            print(f"\r(p={p:5.2e}) Decoding block n. {done:3}/{my_shots:4}... "
                  f"Dec. failure rates (X,Z): {tot['DecFailures_X'] / done:.2e}, "
                  f"{tot['DecFailures_Z'] / done:.2e} ({done / (time.time() - t0):.3g} shots/s)",
                  end="", flush=True)
    if dist is not None and world > 1:
        import torch
        backend = dist.get_backend()
        dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([tot[k] for k in COUNTER_KEYS], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)   # the sweep's only collective
        tot = dict(zip(COUNTER_KEYS, (int(v) for v in t.cpu().tolist())))
    if verbose and rank == 0:
        print()
    return {
        "DecFailures_X": tot["DecFailures_X"],
        "DecFailures_Z": tot["DecFailures_Z"],
        "decSuccessExact": tot["decSuccessExact"],
        "decSuccessDegen": tot["decSuccessDegen"],
        "Avg_number_of_iterations_X": tot["nIterAccX"] / float(shots),
        "Avg_number_of_iterations_Z": tot["nIterAccZ"] / float(shots),
    }


def format_results(p, results, shots):
    """The reference's results table (simulator.py:342-347)."""
    lines = ["\n                             ===          SIMULATION RESULTS          ===\n",
             "   Depolarizing probability | qBlock error rate | Decoding failures (X,Z) | Average iterations (X,Z)",
             "----------------------------+-------------------+-------------------------+---------------------------"]
    for pT, r in zip(p, results):
        qbler = 1. - (r["decSuccessExact"] + r["decSuccessDegen"]) / shots
        lines.append(f"         {pT:10.2e}         |     {qbler:7.2e}      |       "
                     f"{r['DecFailures_X']:5},{r['DecFailures_Z']:5}       |      "
                     f"{r['Avg_number_of_iterations_X']:5.2f}, {r['Avg_number_of_iterations_Z']:5.2f}")
    return "\n".join(lines)


def _load_results(path, meta):
    """Per-p results already in a resumable results file (JSON), if its
    run parameters match `meta`; else empty."""
    import json
    import os
    if not path or not os.path.exists(path):
        return {}
    with open(path) as f:
        doc = json.load(f)
    if doc.get("meta") != meta:
        raise ValueError(f"{path} holds results of a different run: {doc.get('meta')}")
    return {float(k): v for k, v in doc.get("results", {}).items()}


def _save_results(path, meta, done):
    import json
    import os
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump({"meta": meta, "results": {repr(k): v for k, v in sorted(done.items())}}, f, indent=1)
    os.replace(tmp, path)                      # atomic: a killed run leaves the last good file


def simulate(HxFile: str, HzFile: str, p, shots: int = 1000, decType: str = "MS",
             decIterations: int = 99, decSchedule: str = "F", OSDorder: int = -1,
             rngSeed: Optional[int] = None, *, batch_size: Optional[int] = None, verbose: bool = True,
             return_results: bool = False, sampler: Optional[str] = None,
             resultsFile: Optional[str] = None, on_point=None):
    """p-sweep + results table (simulator.py:319-347). Returns None like the
    reference unless return_results=True.

    resultsFile (extension): a JSON file the sweep writes after every
    p-point; a rerun with the same arguments skips the points already there
    (resumable long sweeps). Only rank 0 writes it.
    on_point (extension): called as on_point(pT, result, seconds) after each
    p-point this call computed (bench.py times the sweep's points with it)."""
    Hx = load_matrix(HxFile)
    Hz = load_matrix(HzFile)
    assert max(p) <= 1. and min(p) >= 0.
    _, rank, world = _dist()
    if sampler is None:                       # the resolved shot source is part of the run
        sampler = "device" if (_device_ok() and _channel_ok(Hx, Hz)) else "host"
    meta = {"Hx": HxFile, "Hz": HzFile, "shots": shots, "decType": decType,
            "decIterations": decIterations, "decSchedule": decSchedule, "OSDorder": OSDorder,
            "rngSeed": rngSeed, "world": world, "sampler": sampler}
    done = _load_results(resultsFile, meta)
    results = []
    for pT in p:
        if float(pT) in done:
            results.append(done[float(pT)])
            continue
        t0 = time.perf_counter()
        r = simulate_p(Hx, Hz, p=pT, shots=shots, rngSeed=rngSeed, decType=decType,
                       decIterations=decIterations, decSchedule=decSchedule,
                       OSDorder=OSDorder, batch_size=batch_size, verbose=verbose,
                       sampler=sampler)
        if on_point is not None:
            on_point(pT, r, time.perf_counter() - t0)
        results.append(r)
        done[float(pT)] = r
        if resultsFile and rank == 0:
            _save_results(resultsFile, meta, done)
    if rank == 0:
        print(format_results(p, results, shots))
    return results if return_results else None


def _init_dist_from_env():
    """One process per GPU under torchrun (WORLD_SIZE > 1 in the environment):
    bind this rank to its device and join the process group (RCCL over xGMI;
    QLDPC_SIM_BACKEND=gloo to rehearse on CPU or with ranks sharing a GPU).
    Returns True if this call created the group."""
    import os
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return False
    import torch
    import torch.distributed as dist
    if dist.is_initialized():
        return False
    backend = os.environ.get("QLDPC_SIM_BACKEND", "nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        ndev = torch.cuda.device_count()
        if local >= ndev:
            if backend == "nccl":
                # one process per GPU: under RCCL a second rank on a device is
                # a launch error, not something to fold silently (bench.py too)
                raise RuntimeError(f"LOCAL_RANK {local} but only {ndev} HIP device(s) visible: launch at "
                                   "most one rank per GPU (QLDPC_SIM_BACKEND=gloo rehearses more ranks)")
            local %= max(1, ndev)              # gloo rehearsal: ranks may share a device
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            return True
    dist.init_process_group(backend)
    return True


def main(argv=None):
    parser = argparse.ArgumentParser(description="Stim-based QC-LDPC depolarizing-channel simulator.")
    parser.add_argument("--Hx", required=True, help="Path to Hx parity-check matrix (.npy).")
    parser.add_argument("--Hz", required=True, help="Path to Hz parity-check matrix (.npy).")
    parser.add_argument("--p", type=float, nargs="+", required=True, help="Depolarizing probability.")
    parser.add_argument("--shots", type=int, default=1000, help="Number of Monte Carlo shots.")
    parser.add_argument("--rngSeed", type=int, default=None, help="RNG seed.")
    parser.add_argument("--decType", choices=["NG", "BF", "MS", "BP"], default="MS",
                        help="Decoder type: [NG] Naive Greedy; [MS] Min-Sum; [BP] Belief Propagation.")
    parser.add_argument("--decIterations", type=int, default=99, help="Number of decoding iterations.")
    parser.add_argument("--decSchedule", choices=["F", "L", "S"], default="F",
                        help="Decoder scheduling method: [F] flooding; [L] layered; [S] serial.")
    parser.add_argument("--OSDorder", type=int, default=-1, help="Ordered Statistics Decoding order.")
    parser.add_argument("--batch", type=int, default=None,
                        help="Shots per batch (default on the GPU: 2^20 without OSD, 2^18 with OSD; "
                             "2^16 on the host path).")
    parser.add_argument("--sampler", choices=["device", "host"], default=None,
                        help="Where shots are sampled and counted (default: device if present).")
    parser.add_argument("--results", default=None,
                        help="Resumable results file (JSON, written after every p-point).")
    args = parser.parse_args(argv)
    own_group = _init_dist_from_env()              # torchrun: shots shard over the ranks
    _, rank, _ = _dist()
    if rank == 0:
        print("\n   Command line arguments:")
        print(args)
        print("")
    try:
        simulate(HxFile=args.Hx, HzFile=args.Hz, p=args.p, shots=args.shots, decType=args.decType,
                 decIterations=args.decIterations, decSchedule=args.decSchedule,
                 OSDorder=args.OSDorder, rngSeed=args.rngSeed, batch_size=args.batch,
                 sampler=args.sampler, resultsFile=args.results)
    finally:
        if own_group:
            import torch.distributed as dist
            dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1:])
