"""bench.py — decoded shots/s for qLDPCsim's decode hot path on MI355X.

Headline workload (BASELINE.json metric "decoded shots/sec (MS 50-iter,
LP118_0) at 1/2/4/8 GPU"): LP118_0, normalized min-sum, flooding, max 50
iterations, fixed-work uniform random syndromes (unsatisfiable w.p. >= 255/256,
so every decode runs 50 iterations). One shot = X half (Hz,
sy_z) + Z half (Hx, sy_x); one step = one batch of `--batch` shots per GPU =
two decode kernel launches. Syndromes are generated on the device before
timing (inputs resident in HBM); output buffers are allocated once.

Multi-GPU (weak scaling, no data-path collective; the reference's serial shot
loop simulator.py:244 becomes shards of shots): one process per GPU over RCCL.
  * under torch.distributed.run (WORLD_SIZE set): this process is one rank;
  * `python bench.py --gpus N` with no WORLD_SIZE: spawns N fresh rank
    processes itself (the parent never initialises the GPU).
N larger than the visible devices fails loudly, unless QLDPC_BENCH_BACKEND=gloo
(rehearsal: ranks share devices). The timed region is bracketed by barrier +
synchronize; elapsed time is the max over ranks; `value` = all ranks' shots /
that time.

`roofline` prices the decode kernel against the on-chip unit that binds it
(DESIGN.md §5): VALU issue time by instruction class (a wave64 32-bit VALU op
occupies a SIMD-32 for 2 cycles, a float64 add / mul / fma 4, transcendentals
8 / 16; 1024 SIMDs at 2.4 GHz) or the LDS array (one cycle per CU per LDS
array cycle, 256 CUs at 2.4 GHz). Per-unit
instruction / LDS-cycle / HBM-byte counts come from a committed rocprofv3
profile of the same kernel build (profiles/*_roofline.json, matched by kernel
name and by the hash of the library's device code object), multiplied by this
run's executed half-shot iterations and divided by this run's kernel time (HIP
events on the launch stream). The HBM figures (measured PMC bytes, and
SURVEY.md §8d's algorithmic streaming model) are reported beside it.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
                       [--code C] [--algo MS|BP] [--schedule F|L|S] [--p P] [--iters I]
"""
import argparse
import glob
import hashlib
import json
import os
import re
import shlex
import socket
import struct
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decoded shots/sec (MS 50-iter, LP118_0) at 1/2/4/8 GPU; achieved HBM GB/s"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
CLOCK_GHZ = 2.4                # max engine clock (MI355X_MICROARCH.md)
SIMDS, CUS = 1024, 256         # 256 CUs x 4 SIMDs
VALU_CYCLES = 4                # SQ accounting: one wave64 VALU instruction = one quad-cycle
REFERENCE_PER_CORE = 2.61      # reference decoders.py, LP118_0 MS-F 50 it fixed work, 1 core


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (ranks); default: WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1 << 20, help="shots per GPU per step")
    ap.add_argument("--code", default="LP118_0")
    ap.add_argument("--algo", default="MS", choices=["MS", "BP"])
    ap.add_argument("--schedule", default="F", choices=["F", "L", "S"])
    ap.add_argument("--p", type=float, default=None,
                    help="depolarizing p for channel syndromes (device sampler); default: "
                         "uniform random syndromes (fixed work)")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--io", default="bits", choices=["bits", "bytes"],
                    help="syndrome / hard-decision format in HBM: bit-packed 64-bit words (default) or bytes")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="bounded CPU-baseline sample per leg (0 disables)")
    ap.add_argument("--path", default="auto", choices=["auto", "hbm"],
                    help="hbm: decode through the HBM-resident kernel (library option force_hbm) in the timed region")
    ap.add_argument("--hbm-leg", type=int, default=1,
                    help="N=1: also time the same workload through the HBM-resident kernel (hbm_streaming field)")
    ap.add_argument("--worklog", default=None,
                    help="write per-launch work (kernel, half-shots, iterations) as JSON (profiling)")
    ap.add_argument("--sim-legs", default="3,4",
                    help="end-to-end legs after the headline, comma-separated BASELINE.json config indices "
                         "(3: LP118_2 MS-L + OSD-0 at p = 0.1, strong and per-rank; 4: LP118_2 BP-L, the "
                         "p-sweep [0.01, 0.02, 0.05, 0.1] through simulate), '' for none")
    ap.add_argument("--sim-shots", type=int, default=1 << 20,
                    help="shots of the configs[3] job in total (strong; the per-rank leg: per rank) and of "
                         "each configs[4] p-point in total")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# host facts
# ---------------------------------------------------------------------------
def host_cores():
    """CPU cores this process may use (qldpcsim_amd/hostcores.py): the
    affinity mask, capped by a cgroup CPU quota and by OMP_NUM_THREADS (the
    GPU box sets it to the box's CPU share). Returns (cores, how)."""
    from qldpcsim_amd import hostcores
    return hostcores.process_cores()


def device_code_sha(path):
    """sha256 of the library's embedded device code (the .hip_fatbin ELF
    section): unchanged by host-only edits, changed by any kernel edit."""
    with open(path, "rb") as f:
        data = f.read()
    try:
        shoff, = struct.unpack_from("<Q", data, 0x28)
        shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
        secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
        stroff = secs[shstrndx][4]
        for s in secs:
            nm = data[stroff + s[0]:data.index(b"\0", stroff + s[0])]
            if nm == b".hip_fatbin":
                return hashlib.sha256(data[s[4]:s[4] + s[5]]).hexdigest()
    except (struct.error, ValueError, IndexError):
        pass
    return hashlib.sha256(data).hexdigest()


def _demangle_kernel(sym):
    """'_ZN5qldpc15ms_flood_kernelILi8ELi4EEEvNS_10DecodeArgsE' -> 'ms_flood_kernel<8, 4>'
    (the kernel names rocprofv3 prints for this library's templates: int and
    bool non-type arguments only); '_ZN5qldpc16osd_order_kernelENS_9OrderArgsE'
    -> 'osd_order_kernel'; None for anything else."""
    m = re.match(r"_ZN5qldpc(\d+)", sym)
    if not m:
        return None
    i = m.end()
    name = sym[i:i + int(m.group(1))]
    i += int(m.group(1))
    if sym[i:i + 1] == "E":
        return name
    if sym[i:i + 1] != "I":
        return None
    i += 1
    args = []
    while True:
        a = re.compile(r"L([ib])(n?\d+)E").match(sym, i)
        if not a:
            break
        args.append(("false", "true")[int(a.group(2))] if a.group(1) == "b" else a.group(2).replace("n", "-"))
        i = a.end()
    if sym[i:i + 1] != "E":
        return None
    return f"{name}<{', '.join(args)}>"


def kernel_code_sha(path, kernel):
    """sha256 of one kernel's machine code and kernel descriptor inside the
    library's gfx950 code objects (every offload bundle of .hip_fatbin), so a
    profile stays valid across edits of OTHER kernels; None if not found."""
    with open(path, "rb") as f:
        data = f.read()
    h = None
    pos = 0
    while True:
        pos = data.find(b"__CLANG_OFFLOAD_BUNDLE__", pos)
        if pos < 0:
            break
        n_ent, = struct.unpack_from("<Q", data, pos + 24)
        off = pos + 32
        for _ in range(n_ent):
            eo, esz, tl = struct.unpack_from("<QQQ", data, off)
            triple = data[off + 24:off + 24 + tl]
            off += 24 + tl
            if b"gfx950" not in triple or esz == 0:
                continue
            elf = data[pos + eo:pos + eo + esz]
            shoff, = struct.unpack_from("<Q", elf, 0x28)
            shentsize, shnum, _ = struct.unpack_from("<HHH", elf, 0x3A)
            secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
            for s in secs:
                if s[1] != 2:                                  # SHT_SYMTAB
                    continue
                strtab = secs[s[6]]
                for j in range(s[5] // 24):
                    st_name, st_info, _, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", elf, s[4] + j * 24)
                    nm = elf[strtab[4] + st_name:elf.index(b"\0", strtab[4] + st_name)].decode()
                    if (st_info & 0xf) != 2 or _demangle_kernel(nm) != kernel:     # STT_FUNC
                        continue
                    h = hashlib.sha256()
                    tsec = secs[st_shndx]
                    h.update(elf[tsec[4] + st_value - tsec[3]:tsec[4] + st_value - tsec[3] + st_size])
                    for k in range(s[5] // 24):                # its kernel descriptor (<sym>.kd)
                        kn, _, _, ksh, kv, ksz = struct.unpack_from("<IBBHQQ", elf, s[4] + k * 24)
                        if elf[strtab[4] + kn:elf.index(b"\0", strtab[4] + kn)] == (nm + ".kd").encode():
                            ks = secs[ksh]
                            h.update(elf[ks[4] + kv - ks[3]:ks[4] + kv - ks[3] + ksz])
                    return h.hexdigest()
        pos += 24
    return None


WORKLOAD_KEYS = ("code", "algo", "schedule", "p", "iters")


def workload_of(args):
    """The workload a profile entry's counters depend on (not the batch size or
    the step counts): code, decoder, schedule, channel p, iteration cap."""
    return {k: getattr(args, k) for k in WORKLOAD_KEYS}


def _profile_order(path):
    """Newest first without trusting the tag's spelling: round number, then
    the tag's letter sequence as a bijective base-26 count (r04z < r04aa),
    then any variant suffix."""
    tag = os.path.basename(path).split("_")[0]
    m = re.match(r"r(\d+)([a-z]*)", tag)
    if not m:
        return (0, 0, tag)
    rnd, letters = int(m.group(1)), m.group(2)
    seq = 0
    for ch in letters:
        seq = seq * 26 + (ord(ch) - 96)
    return (rnd, seq, tag)


def find_profile(kernel, sha, code_sha=None, workload=None):
    """Newest profiles/*_roofline.json entry for this kernel built from this
    device code: the kernel's own machine-code hash (`code_sha256` of the
    entry) when both sides have it, else the whole device image's (None if the
    committed profiles are stale for this build). With `workload`
    (workload_of(args)), an entry whose `bench_args` ran the same workload is
    preferred — the per-iteration counts of one kernel differ between codes,
    channel p and schedules; a build match of another workload is returned only
    when no entry ran this one, flagged `workload_match: False`."""
    other = (None, None)
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_roofline.json")), key=_profile_order, reverse=True)
    for path in paths:
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        for k in d.get("kernels", []):
            if k.get("kernel") != kernel:
                continue
            if code_sha is not None and k.get("code_sha256") is not None:
                if k["code_sha256"] != code_sha:
                    continue
            elif d.get("device_code_sha256") != sha:
                continue
            if workload is None:
                return os.path.relpath(path, ROOT), k
            try:
                ran = workload_of(parse(shlex.split(k.get("bench_args", ""))))
            except SystemExit:
                ran = None
            if ran == workload:
                return os.path.relpath(path, ROOT), dict(k, workload_match=True)
            if other[0] is None:
                other = (os.path.relpath(path, ROOT), dict(k, workload_match=False))
    return other


# ---------------------------------------------------------------------------
# algorithmic byte model — reported beside the roofline
# ---------------------------------------------------------------------------
def algorithmic_bytes_per_iter(H, layer_ptr, layer_rows, word):
    """Bytes one executed iteration of one half-shot moves under the HBM
    streaming model: flooding w(3E + 2n); layered sum over layers of
    w(2E_l + sum_{j in V_l} d_j + 2|V_l|)."""
    m, n = H.shape
    E = int(H.sum())
    if len(layer_ptr) == 2 and layer_ptr[1] == m:
        return word * (3 * E + 2 * n)
    deg = H.sum(axis=0)
    tot = 0
    for l in range(len(layer_ptr) - 1):
        rows = layer_rows[layer_ptr[l]:layer_ptr[l + 1]]
        El = int(H[rows].sum())
        V = np.flatnonzero(H[rows].any(axis=0))
        tot += word * (2 * El + int(deg[V].sum()) + 2 * len(V))
    return tot


def structural_bytes_per_iter(H, layer_ptr, layer_rows, word):
    """What hbm_tile_kernel itself moves per executed half-shot iteration:
    the §8(d) model plus one column-sum read per edge (the exact check node
    needs S_j and c2v_e on every edge): flooding w(4E + 2n)."""
    m, _ = H.shape
    if len(layer_ptr) == 2 and layer_ptr[1] == m:
        e_sched = int(H.sum())
    else:
        e_sched = sum(int(H[layer_rows[layer_ptr[l]:layer_ptr[l + 1]]].sum()) for l in range(len(layer_ptr) - 1))
    return algorithmic_bytes_per_iter(H, layer_ptr, layer_rows, word) + word * e_sched


# ---------------------------------------------------------------------------
# CPU baselines (rank 0, N = 1): bounded samples of the same workload
# ---------------------------------------------------------------------------
def _cpu_syndromes(Hx, Hz, p, B, rng):
    if p is None:
        return (rng.integers(0, 2, (B, Hz.shape[0]), dtype=np.uint8),
                rng.integers(0, 2, (B, Hx.shape[0]), dtype=np.uint8))
    from qldpcsim_amd.simulator import sample_channel
    sz, sx, _, _ = sample_channel(Hx, Hz, p, B, rng)
    return sz, sx


def cpu_baseline_port(args, cores):
    """oracle/qldpc_oracle.c (OpenMP over shots, bit-exact vs the reference's
    golden vectors) on `cores` threads."""
    from oracle import oracle
    from qldpcsim_amd import codes, schedule
    Hx, Hz = codes.load_code(args.code)
    lx, lz = schedule.select_layers(Hx, Hz, args.schedule)
    (lpx, lrx), (lpz, lrz) = schedule.pack_layers(lx, Hz.shape[0]), schedule.pack_layers(lz, Hx.shape[0])
    prior = (0.05 if args.p is None else args.p) / 3
    rng = np.random.default_rng(12345)
    chunk = 64 * cores
    shots = 0
    t0 = time.perf_counter()
    while True:
        sz, sx = _cpu_syndromes(Hx, Hz, args.p, chunk, rng)
        oracle.decode_batch(args.algo, Hz, sz, prior, args.iters, lpx, lrx, want_post=False, nthreads=cores)
        oracle.decode_batch(args.algo, Hx, sx, prior, args.iters, lpz, lrz, want_post=False, nthreads=cores)
        shots += chunk
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds:
            break
    return {"value": shots / el, "unit": "shots/s", "cores": cores, "kind": "port",
            "sample": f"{shots} shots of the bench workload (both halves) in {el:.1f} s with "
                      f"oracle/qldpc_oracle.c, {cores} OpenMP threads"}


def _numpy_worker(a):
    code, sched, p, iters, seconds, seed = a
    from oracle import numpy_dense
    from qldpcsim_amd import codes, schedule
    Hx, Hz = codes.load_code(code)
    lx, lz = schedule.select_layers(Hx, Hz, sched)
    dz, dx = numpy_dense.DenseMinSum(Hz), numpy_dense.DenseMinSum(Hx)
    prior = (0.05 if p is None else p) / 3
    rng = np.random.default_rng(seed)
    shots = 0
    t0 = time.perf_counter()
    while True:
        sz, sx = _cpu_syndromes(Hx, Hz, p, 1, rng)
        dz.decode(sz[0].astype(np.int64), prior, iters, lx)
        dx.decode(sx[0].astype(np.int64), prior, iters, lz)
        shots += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return shots, el


def cpu_baseline_numpy(args, cores):
    """oracle/numpy_dense.py (the reference's dense per-shot structure,
    bit-exact vs its golden vectors): one process per core, OMP_NUM_THREADS=1."""
    import multiprocessing as mp
    old = os.environ.get("OMP_NUM_THREADS")
    os.environ["OMP_NUM_THREADS"] = "1"
    try:
        with mp.get_context("spawn").Pool(cores) as pool:
            res = pool.map(_numpy_worker, [(args.code, args.schedule, args.p, args.iters,
                                            args.cpu_seconds, 777 + i) for i in range(cores)])
    finally:
        if old is None:
            os.environ.pop("OMP_NUM_THREADS", None)
        else:
            os.environ["OMP_NUM_THREADS"] = old
    rate = sum(s / e for s, e in res)
    tot = sum(s for s, _ in res)
    return {"value": rate, "unit": "shots/s", "cores": cores, "kind": "port",
            "sample": f"{tot} shots one at a time over {cores} processes, ~{args.cpu_seconds:.0f} s each, "
                      f"oracle/numpy_dense.py (dense NumPy restatement of decoders.py:147-177)"}


def cpu_baselines(args):
    cores, how = host_cores()
    legs = [cpu_baseline_port(args, cores)]
    if args.algo == "MS":
        legs.append(cpu_baseline_numpy(args, cores))
    out = dict(legs[0])
    out["cores_source"] = how
    out["legs"] = legs
    if args.code == "LP118_0" and args.algo == "MS" and args.schedule == "F" and args.p is None:
        out["reference_context"] = {
            "value": REFERENCE_PER_CORE, "unit": "shots/s/core",
            "source": "the reference's own decoders.py on this workload, 1 core (BASELINE.md survey run)",
            "x_cores": REFERENCE_PER_CORE * cores}
    return out


# ---------------------------------------------------------------------------
# end-to-end legs: BASELINE.json configs[3] / configs[4] as they are stated
# ---------------------------------------------------------------------------
SIM_LEGS = {
    3: dict(code="LP118_2", decType="MS", decSchedule="L", OSDorder=0, decIterations=50, p=0.1,
            config="BASELINE.json configs[3]: LP118_2, MS layered + OSD-0, a fixed total of shots sharded "
                   "across the GPUs (strong scaling), p = 0.1"),
    4: dict(code="LP118_2", decType="BP", decSchedule="L", OSDorder=4, decIterations=100,
            p=[0.01, 0.02, 0.05, 0.1],
            config="BASELINE.json configs[4]: LP118_2, BP layered + OSD order 4 (simulate never passes "
                   "OSDorder to BP_decoder, simulator.py:281-282), the p-sweep [0.01, 0.02, 0.05, 0.1] "
                   "through simulate's own p loop (simulator.py:335), a fixed total of shots per p-point "
                   "sharded across the GPUs"),
}


def _sync(dist):
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except ImportError:
        pass
    if dist is not None:
        dist.barrier()


def _gather(dist, world, me):
    if dist is None or world == 1:
        return [me]
    ranks = [None] * world
    dist.all_gather_object(ranks, me)
    return ranks


def sim_leg(idx, shots, dist=None, warmup_shots=1 << 18, sampler=None, per_rank=False):
    """configs[3] end to end through the drop-in simulate_p (reference
    simulator.py:167-315): device sampler, decode, OSD, device counters. The
    job is `shots` shots in total, each rank its contiguous share (strong
    scaling, BASELINE's "1e6 shots sharded across 8 MI355X"); per_rank=True
    gives every rank `shots` of its own instead (weak scaling). simulate_p
    all-reduces the six counters (its only collective). Timed between
    barriers + device syncs, max over ranks."""
    from qldpcsim_amd import codes, decoders, hostcores, simulator
    leg = SIM_LEGS[idx]
    world = dist.get_world_size() if dist is not None else 1
    total = world * shots if per_rank else shots
    Hx, Hz = codes.load_code(leg["code"])
    kw = dict(decType=leg["decType"], decIterations=leg["decIterations"], decSchedule=leg["decSchedule"],
              OSDorder=leg["OSDorder"], verbose=False, sampler=sampler)
    if warmup_shots:
        simulator.simulate_p(Hx, Hz, leg["p"], shots=world * min(warmup_shots, max(1, total // world)),
                             rngSeed=2, **kw)
    decoders.reset_osd_stats()
    _sync(dist)
    t0 = time.perf_counter()
    r = simulator.simulate_p(Hx, Hz, leg["p"], shots=total, rngSeed=1, **kw)
    _sync(dist)
    mine = time.perf_counter() - t0
    st = dict(decoders.OSD_STATS)
    rank = dist.get_rank() if dist is not None else 0
    my_shots = total // world + (1 if rank < total % world else 0)
    me = {"shots": my_shots, "elapsed_s": mine, "shots_per_s": my_shots / mine, "host_cores": hostcores.rank_cores(),
          "osd_shots": st["osd_shots"], "host_order_shots": st["host_order_shots"]}
    ranks = _gather(dist, world, me)
    el = max(x["elapsed_s"] for x in ranks)
    osd = sum(x["osd_shots"] for x in ranks)
    host = sum(x["host_order_shots"] for x in ranks)
    return {"config": leg["config"], "code": leg["code"], "decType": leg["decType"],
            "decSchedule": leg["decSchedule"], "OSDorder": leg["OSDorder"], "decIterations": leg["decIterations"],
            "p": leg["p"], "scaling": "weak" if per_rank else "strong", "shots": total, "n_ranks": world,
            "value": total / el, "unit": "shots/s", "elapsed_s": el, "per_rank": ranks, "osd_shots": osd,
            "host_order_shots": host, "host_order_share": host / osd if osd else 0.0,
            "qBLER": 1.0 - (r["decSuccessExact"] + r["decSuccessDegen"]) / total, "counters": r,
            "timing": "simulate_p between barrier + device sync, max over ranks; counters all-reduced "
                      "inside simulate_p (one all_reduce(SUM) of six int64)"}


def sim_sweep_leg(idx, shots, dist=None, warmup_shots=1 << 16, sampler=None):
    """configs[4]'s qBLER curve end to end through the drop-in simulate
    (reference simulator.py:319-347) and its own p loop (:335): `shots` shots
    per p-point in total, each rank its share, the six counters all-reduced
    per point inside simulate_p. The whole sweep is timed between barriers +
    device syncs (max over ranks); each point by simulate's on_point hook
    (its all-reduce ends every point on all ranks together; max over ranks)."""
    import contextlib
    import tempfile
    from qldpcsim_amd import codes, hostcores, simulator
    leg = SIM_LEGS[idx]
    world = dist.get_world_size() if dist is not None else 1
    Hx, Hz = codes.load_code(leg["code"])
    tmp = tempfile.mkdtemp(prefix="qldpc_bench_")
    fx, fz = os.path.join(tmp, "Hx.npy"), os.path.join(tmp, "Hz.npy")
    np.save(fx, Hx)
    np.save(fz, Hz)
    kw = dict(decType=leg["decType"], decIterations=leg["decIterations"], decSchedule=leg["decSchedule"],
              OSDorder=leg["OSDorder"], verbose=False, sampler=sampler)
    if warmup_shots:
        simulator.simulate_p(Hx, Hz, max(leg["p"]), shots=world * warmup_shots, rngSeed=2, **kw)
    points = []
    _sync(dist)
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(sys.stderr):         # simulate's results table: not bench's JSON line
        res = simulator.simulate(fx, fz, leg["p"], shots=shots, rngSeed=1, return_results=True,
                                 on_point=lambda pT, r, sec: points.append(sec), **kw)
    _sync(dist)
    mine = time.perf_counter() - t0
    for f in (fx, fz):
        os.remove(f)
    os.rmdir(tmp)
    ranks = _gather(dist, world, {"elapsed_s": mine, "points_s": points, "host_cores": hostcores.rank_cores()})
    el = max(x["elapsed_s"] for x in ranks)
    curve = []
    for i, (pT, r) in enumerate(zip(leg["p"], res)):
        sec = max(x["points_s"][i] for x in ranks)
        curve.append({"p": pT, "shots": shots, "elapsed_s": sec, "value": shots / sec, "unit": "shots/s",
                      "qBLER": 1.0 - (r["decSuccessExact"] + r["decSuccessDegen"]) / shots, "counters": r})
    return {"config": leg["config"], "code": leg["code"], "decType": leg["decType"],
            "decSchedule": leg["decSchedule"], "OSDorder": leg["OSDorder"], "decIterations": leg["decIterations"],
            "p": leg["p"], "scaling": "strong", "shots_per_point": shots, "n_ranks": world,
            "value": shots * len(leg["p"]) / el, "unit": "shots/s (whole sweep)", "elapsed_s": el,
            "curve": curve, "per_rank": [{"elapsed_s": x["elapsed_s"], "points_s": x["points_s"],
                                          "host_cores": x["host_cores"]} for x in ranks],
            "timing": "simulate(p=[...]) between barrier + device sync, max over ranks; per point: "
                      "simulate's on_point hook, max over ranks; counters all-reduced per point"}


def sim_legs(args, dist, world):
    """The end-to-end legs bench.py runs after the headline (--sim-legs)."""
    legs = [int(x) for x in args.sim_legs.split(",") if x.strip()]
    out = {}
    if 3 in legs:
        strong = sim_leg(3, args.sim_shots, dist)
        if world == 1:
            weak = dict(strong, scaling="weak", note="at one GPU the per-rank job is the whole job: "
                                                     "the same run as the strong leg")
        else:
            weak = sim_leg(3, args.sim_shots, dist, per_rank=True)
        out["configs3"] = dict(strong, weak_per_rank=weak)
    if 4 in legs:
        out["configs4"] = sim_sweep_leg(4, args.sim_shots, dist)
    return out


# ---------------------------------------------------------------------------
# one rank
# ---------------------------------------------------------------------------
def run_rank(args, rank, world, local):
    import torch
    import torch.distributed as dist

    backend = os.environ.get("QLDPC_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if ndev == 0:
        raise SystemExit("bench.py: no HIP device visible")
    if local >= ndev and backend == "nccl":
        raise SystemExit(f"bench.py: rank {rank} has local rank {local} but only {ndev} device(s) are "
                         "visible (one GPU per rank; QLDPC_BENCH_BACKEND=gloo to rehearse on shared devices)")
    cpu = None
    if world == 1 and rank == 0 and args.cpu_seconds > 0:
        cpu = cpu_baselines(args)          # before the GPU is touched (spawned pool)
    dev = torch.device("cuda", local % ndev)
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from qldpcsim_amd import _lib, codes, decoders, schedule
    if args.path == "hbm":
        _lib.set_option("force_hbm", 1)
    from qldpcsim_amd.simulator import DeviceChannel
    Hx, Hz = codes.load_code(args.code)
    m, n = Hz.shape
    E = int(Hz.sum())
    lx, lz = schedule.select_layers(Hx, Hz, args.schedule)
    lpx, lrx = schedule.pack_layers(lx, Hz.shape[0])       # X half: Hz with Hx's layers
    lpz, lrz = schedule.pack_layers(lz, Hx.shape[0])       # Z half: Hx with Hz's layers
    B = args.batch
    if args.p is None:
        g = torch.Generator(device=dev).manual_seed(20251226 + rank)
        syn_z = torch.randint(0, 2, (B, Hz.shape[0]), dtype=torch.uint8, device=dev, generator=g)
        syn_x = torch.randint(0, 2, (B, Hx.shape[0]), dtype=torch.uint8, device=dev, generator=g)
        prior = 0.05 / 3
    else:
        ch = DeviceChannel(Hx, Hz, dev, seed=20251226 + rank)
        syn_z, syn_x, _, _ = ch.sample(args.p, B)
        prior = args.p / 3
    bits = args.io == "bits"
    if bits:                                             # the wire format of SURVEY 8f-4
        syn_z, syn_x = decoders.pack_bits(syn_z), decoders.pack_bits(syn_x)
    halves = ((Hz, syn_z, lpx, lrx), (Hx, syn_x, lpz, lrz))
    want_post = False

    def buffers(H):
        eshape = (B, (H.shape[1] + 63) // 64) if bits else (B, H.shape[1])
        return decoders.DecodeResult(torch.empty(eshape, dtype=torch.int64 if bits else torch.uint8, device=dev),
                                     torch.empty(B, dtype=torch.int32, device=dev), None,
                                     torch.empty(B, dtype=torch.int32, device=dev))
    outs = [buffers(H) for H, _, _, _ in halves]

    log = []                                               # per launch: (kernel, half-shots, iters tensor)
    names = [_lib.kernel_name(H, lp, lr, args.algo, dev.index) for H, _, lp, lr in halves]

    def step():
        res = []
        for (H, s, lp, lr), o, nm in zip(halves, outs, names):
            r = decoders.decode_batch(H, s, prior, args.iters, algo=args.algo, out=o, layer_ptr=lp,
                                      layer_rows=lr, want_post=want_post, ehat_bits=bits)
            res.append(r)
            if args.worklog:
                log.append((nm, B, r.iters.sum(dtype=torch.int64)))
        return res

    iters_sum = torch.zeros((), dtype=torch.int64, device=dev)
    for _ in range(args.warmup):
        # the same work as a timed step, including the iteration reduction (the
        # first use of torch's reduce kernel loads its code object: ~0.1 s)
        for r in step():
            iters_sum += r.iters.sum(dtype=torch.int64)
    torch.cuda.synchronize()
    _lib.timing_enable(True)
    _lib.timing_reset()
    iters_sum.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for r in step():
            iters_sum += r.iters.sum(dtype=torch.int64)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms, launches = _lib.timing_read()
    _lib.timing_enable(False)
    if world > 1:
        tdev = dev if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if args.worklog and rank == 0:
        with open(args.worklog, "w") as f:
            json.dump({"launches": [{"kernel": nm, "half_shots": b, "iters": int(it.item())}
                                    for nm, b, it in log]}, f)
    total_shots = B * args.steps * world
    value = total_shots / elapsed

    halves_timed = 2 * B * args.steps
    its = int(iters_sum.item())
    avg_launch_s = kern_ms / 1e3 / launches
    hs_per_launch = halves_timed / launches
    it_per_launch = its / launches
    word = 4 if args.algo == "MS" else 8
    algo_bytes = sum(algorithmic_bytes_per_iter(H.astype(np.int64), lp, lr, word) for H, _, lp, lr in halves) / 2
    io_bytes = 8 * ((m + 63) // 64 + (n + 63) // 64) + 4 if bits else m + n + 4
    algo_launch = algo_bytes * it_per_launch + io_bytes * hs_per_launch
    roof = roofline(names, avg_launch_s, hs_per_launch, it_per_launch, algo_launch, launches, workload_of(args))
    try:                                   # launch geometry (older library builds lack the call)
        H0, _, lp0, lr0 = halves[0]
        w, b, lds = _lib.launch_info(H0, lp0, lr0, args.algo, dev.index)
        roof["occupancy"] = {"waves_per_workgroup": w, "workgroups_per_cu": b, "waves_per_cu": w * b,
                             "lds_bytes_per_workgroup": lds}
    except (AttributeError, RuntimeError, ValueError):
        pass

    hbm_leg = None
    if world == 1 and args.hbm_leg and not args.worklog and args.path != "hbm":
        hbm_leg = hbm_streaming_leg(halves, outs, prior, args, B, bits, algo_launch, dev)

    sched_name = {"F": "flooding", "L": "layered", "S": "serial"}[args.schedule]
    algo_name = "normalized min-sum (beta 0.75)" if args.algo == "MS" else "sum-product BP"
    synd = "fixed-work uniform random syndromes (SURVEY.md 8d(i))" if args.p is None else \
        f"depolarizing channel p={args.p} (device Philox sampler)"
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "shots/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32+f64" if args.algo == "MS" else "f64",
        "data": "synthetic",
        "config": {
            "workload": f"{args.code} {algo_name}, {sched_name}, max {args.iters} iterations, {synd}; "
                        "1 shot = X half + Z half",
            "code": args.code, "algo": args.algo, "schedule": args.schedule, "p": args.p,
            "m": m, "n": n, "edges": E,
            "shots_per_gpu_per_step": B, "global_batch": B * world,
            "avg_iterations": its / halves_timed,
            "io": "syndromes and hard decisions bit-packed (64-bit words)" if bits else "one byte per bit",
            "parallelism": f"shots sharded over {world} GPU(s) (one process per GPU, {backend}), "
                           "no data-path collective",
        },
        "roofline": roof,
        "parity_pin": {k: v for k, v in decoders.parity_pins().items()},
    }
    if hbm_leg is not None:
        out["hbm_streaming"] = hbm_leg
    if args.sim_legs.strip() and not args.worklog:
        out["simulate"] = sim_legs(args, dist if world > 1 else None, world)
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def hbm_streaming_leg(halves, outs, prior, args, B, bits, algo_launch, dev, steps=2):
    """The same workload through hbm_tile_kernel (message state in HBM, every
    message a coalesced 256-byte tile row; option force_hbm): SURVEY.md
    §8(d)'s HBM roofline is the bound of that design. Reported beside the
    headline (which is the LDS-resident kernel's), untimed by the headline."""
    import torch
    from qldpcsim_amd import _lib, decoders
    with _lib.options(force_hbm=1):
        name = _lib.kernel_name(halves[0][0], halves[0][2], halves[0][3], args.algo, dev.index)

        def step():
            for (H, s, lp, lr), o in zip(halves, outs):
                decoders.decode_batch(H, s, prior, args.iters, algo=args.algo, out=o, layer_ptr=lp,
                                      layer_rows=lr, want_post=False, ehat_bits=bits)
        step()
        torch.cuda.synchronize()
        _lib.timing_enable(True)
        _lib.timing_reset()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kern_ms, launches = _lib.timing_read()
        _lib.timing_enable(False)
    t_launch = kern_ms / 1e3 / launches
    gbs = algo_launch / t_launch / 1e9
    H0, _, lp0, lr0 = halves[0]
    w = 8 if args.algo == "BP" else 4
    struct = structural_bytes_per_iter(H0, lp0, lr0, w) / algorithmic_bytes_per_iter(H0, lp0, lr0, w)
    measured = None
    _, prof = find_profile(name, None, kernel_code_sha(_lib.LIB_PATH, name))
    if prof is not None:                               # PMC bytes per half-shot of this kernel build
        measured = prof["per_half_shot"]["hbm_bytes"] * (2 * B * steps / launches) / t_launch / 1e9
    return {"kernel": name, "value": B * steps / el, "unit": "shots/s", "steps": steps,
            "measured_gbs": measured, "measured_frac": None if measured is None else measured / HBM_PEAK_GBS,
            "kernel_ms_per_launch": t_launch * 1e3, "algorithmic_gbs": gbs, "peak_gbs": HBM_PEAK_GBS,
            "frac": gbs / HBM_PEAK_GBS,
            "structural_over_model": struct, "structural_gbs": gbs * struct,
            "note": "the same workload and iteration counts through the HBM-resident decoder "
                    "(option force_hbm); GB/s under SURVEY.md 8d's algorithmic model; the kernel's "
                    "structural bytes (structural_gbs) add one column-sum read per edge, the floor of an "
                    "exact check node (DESIGN.md 3.6); the headline value is the LDS-resident kernel's"}


def roofline(names, t_launch, hs_launch, it_launch, algo_launch, launches, workload=None):
    """The bound of the dominant decode kernel (both halves use the same kernel
    on the bundled codes, whose Hx and Hz share a shape), priced with the
    counters of the same kernel build on the same workload."""
    from qldpcsim_amd import _lib
    kernel = names[0]
    sha = device_code_sha(_lib.LIB_PATH)
    ksha = kernel_code_sha(_lib.LIB_PATH, kernel)
    src, prof = find_profile(kernel, sha, ksha, workload)
    r = {"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
         "kernel": kernel, "kernel_ms_per_launch": t_launch * 1e3, "launches": launches,
         "units_per_launch": {"half_shots": hs_launch, "half_shot_iterations": it_launch},
         "hbm": {"algorithmic_bytes_per_launch": algo_launch,
                 "algorithmic_gbs": algo_launch / t_launch / 1e9,
                 "algorithmic_model": "SURVEY.md 8d: per executed half-shot iteration w(3E+2n) flooding "
                                      "(layered: sum_l w(2E_l + sum_{V_l} d_j + 2|V_l|)), w = 4 MS / 8 BP, "
                                      "+ I/O bytes per half-shot (m+n+4, or 8(ceil(m/64)+ceil(n/64))+4 bit-packed); "
                                      + ("an HBM-streaming design's bytes, not what this LDS-resident kernel moves"
                                         if not kernel.startswith("hbm_tile") else
                                         "this HBM-resident kernel moves about 1.28x these bytes (post and c2v "
                                         "rows both read per edge)"),
                 "peak_gbs": HBM_PEAK_GBS},
         "device_code_sha256": sha, "kernel_code_sha256": ksha, "profile": src,
         "profile_bench_args": None if prof is None else prof.get("bench_args"),
         "profile_workload_match": None if prof is None else prof.get("workload_match")}
    if prof is None:
        r["note"] = ("no counter profile under profiles/ for this kernel build "
                     "(tools/gpu_profile_roofline.sh regenerates it): bound and frac unmeasured")
        return r
    pu = prof["per_half_shot_iteration"]
    valu_lo = None
    if "valu_cycles" in pu:
        # VALU issue time by instruction class (32-bit ops 2 cycles per wave64
        # on a SIMD-32, float64 add/mul/fma 4, transcendentals 8/16), per SIMD;
        # the unclassified remainder (float64 min/max/compare among them) at
        # the float64 rate: an upper bound, the lower one beside it
        valu = pu.get("valu_cycles_hi", pu["valu_cycles"]) * it_launch / t_launch / 1e9   # G SIMD-cycles / s
        valu_lo = pu["valu_cycles"] * it_launch / t_launch / 1e9
        valu_peak = SIMDS * CLOCK_GHZ
        valu_unit = "G SIMD VALU-issue cycles/s (class-weighted, upper bound)"
    else:
        valu = pu["valu_insts"] * it_launch / t_launch / 1e9             # G wave-instructions / s
        valu_peak = SIMDS * CLOCK_GHZ / VALU_CYCLES
        valu_unit = "G VALU wave-instructions/s (4 cycles each)"
    # LDS: array cycles plus the stores' extra transfer cycles when the
    # profile has the store counts (path cycles, MI355X_MICROARCH.md §LDS:
    # ds_write_b32 4 / b64 6 cycles against 2 / 4 array cycles)
    lds_cyc = pu.get("lds_path_cycles", pu["lds_cycles"])
    lds = lds_cyc * it_launch / t_launch / 1e9                       # G LDS cycles / s (chip)
    lds_array = pu["lds_cycles"] * it_launch / t_launch / 1e9
    lds_peak = CUS * CLOCK_GHZ
    traffic = prof["per_half_shot"]["hbm_bytes"] * hs_launch
    hbm_gbs = traffic / t_launch / 1e9                                # measured (PMC) HBM bytes
    units = {"valu": {"achieved": valu, "peak": valu_peak, "unit": valu_unit,
                      "frac": valu / valu_peak,
                      "frac_lo": None if valu_lo is None else valu_lo / valu_peak},
             "lds": {"achieved": lds, "peak": lds_peak,
                     "unit": ("G LDS cycles/s (all CUs): array + store transfer" if "lds_path_cycles" in pu
                              else "G LDS-array cycles/s (all CUs)"),
                     "frac": lds / lds_peak, "frac_array": lds_array / lds_peak},
             "hbm": {"achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s (measured HBM bytes)",
                     "frac": hbm_gbs / HBM_PEAK_GBS}}
    bound = max(units, key=lambda k: units[k]["frac"])
    r.update(bound=bound, achieved=units[bound]["achieved"], peak=units[bound]["peak"],
             unit=units[bound]["unit"], frac=units[bound]["frac"], traffic=traffic, units=units)
    r["hbm"].update(achieved_gbs=traffic / t_launch / 1e9, frac=traffic / t_launch / 1e9 / HBM_PEAK_GBS)
    r["formula"] = ("valu frac = valu_cycles/half-shot-iter x iterations/launch / (1024 SIMDs x 2.4 GHz x "
                    "launch time), valu_cycles = 2 x SQ_INSTS_VALU + 2 x (ADD+MUL+FMA_F64) + 14 x TRANS_F64 + "
                    "6 x TRANS_F32 (per-class SQ_INSTS_VALU_* counters) + 2 x the unclassified rest "
                    "(float64 min/max/compare have no class counter; frac_lo leaves it out); lds frac = (SQ_LDS_IDX_ACTIVE + 2 x "
                    "SQ_INSTS_LDS_STORE: array + store transfer cycles)/half-shot-iter x "
                    "iterations/launch / (256 CUs x 2.4 GHz x launch time); hbm frac = PMC HBM bytes/half-shot x "
                    "half-shots/launch / launch time / 8000 GB/s; bound = the largest; per-unit counts from the "
                    "profile (SQ_INSTS_VALU, SQ_LDS_IDX_ACTIVE; traffic = 2 x FETCH_SIZE + WRITE_SIZE), "
                    "launch time and iterations from this run")
    r["profile_clock_ghz"] = prof.get("clock_ghz")
    return r


# ---------------------------------------------------------------------------
# launcher
# ---------------------------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawned_rank(rank, world, port, argv):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    run_rank(parse(argv), rank, world, rank)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            raise SystemExit(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world}")
        run_rank(args, int(os.environ.get("RANK", "0")), world, int(os.environ.get("LOCAL_RANK", "0")))
        return
    world = args.gpus or 1
    if world < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if world == 1:
        run_rank(args, 0, 1, 0)
        return
    # N ranks, no launcher: spawn N fresh processes (this one never touches the
    # GPU; device_count does not initialise it on this image)
    import torch
    import multiprocessing as mp
    backend = os.environ.get("QLDPC_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if world > ndev and backend == "nccl":
        raise SystemExit(f"bench.py: --gpus {world} but {ndev} HIP device(s) visible (one GPU per rank; "
                         "set QLDPC_BENCH_BACKEND=gloo to rehearse with ranks sharing devices)")
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_spawned_rank, args=(r, world, port, argv)) for r in range(world)]
    for p in procs:
        p.start()
    rc = 0
    for p in procs:
        p.join()
        rc = rc or (p.exitcode or 0)
    if rc:
        raise SystemExit(f"bench.py: a rank exited with status {rc}")


if __name__ == "__main__":
    main()
