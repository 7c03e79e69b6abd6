"""Multi-process path of the batched simulator on CPU (gloo, world_size 2):
shots shard contiguously across ranks and the six counters are summed with one
all_reduce — results equal the single-process run. The GPU decode is replaced
by the CPU oracle here (tests only); on the GPU node the same code runs over
RCCL with the HIP kernels."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_decode_batch(H, syndromes, p, max_iter, layers=None, algo="MS", beta=0.75, eps=1e-9,
                         want_post=False, osd_order=-1, layer_ptr=None, layer_rows=None, stream=None):
    from oracle import oracle
    from qldpcsim_amd.decoders import DecodeResult
    e, it, post, fl = oracle.decode_batch(algo, H, syndromes, p, max_iter, layer_ptr, layer_rows,
                                          beta=beta, eps=eps, nthreads=1)
    conv = np.all(((e.astype(np.int64) @ np.asarray(H, np.int64).T) % 2) == syndromes, axis=1)
    return DecodeResult(e, it, post if want_post else None, conv.astype(np.int32))


def _samples(shots):
    from qldpcsim_amd import codes
    from qldpcsim_amd.simulator import sample_channel
    Hx, Hz = codes.load_code("LP04_0")
    return Hx, Hz, sample_channel(Hx, Hz, 0.1, shots, np.random.default_rng(99))


def _worker(rank, world, port, shots, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from qldpcsim_amd import decoders, simulator
    decoders.decode_batch = _oracle_decode_batch
    Hx, Hz, smp = _samples(shots)
    res = simulator.simulate_p(Hx, Hz, 0.1, shots=shots, decIterations=20, decSchedule="L",
                               samples=smp, batch_size=17, verbose=False)
    out[rank] = res
    dist.destroy_process_group()


def test_two_rank_gloo_counters_equal_single_process():
    shots = 101                                        # uneven split: 51 + 50
    from qldpcsim_amd import decoders, simulator
    orig = decoders.decode_batch
    decoders.decode_batch = _oracle_decode_batch
    try:
        Hx, Hz, smp = _samples(shots)
        single = simulator.simulate_p(Hx, Hz, 0.1, shots=shots, decIterations=20, decSchedule="L",
                                      samples=smp, batch_size=17, verbose=False)
    finally:
        decoders.decode_batch = orig
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), shots, out), nprocs=2, join=True)
    assert out[0] == single and out[1] == single
    assert single["decSuccessExact"] > 0 and single["Avg_number_of_iterations_X"] > 1.0


def _oracle_decode_batch_osd(H, syndromes, p, max_iter, layers=None, algo="MS", beta=0.75, eps=1e-9,
                             want_post=False, osd_order=-1, layer_ptr=None, layer_rows=None, stream=None):
    from qldpcsim_amd import decoders
    r = _oracle_decode_batch(H, syndromes, p, max_iter, layers, algo, beta, eps, True, -1, layer_ptr, layer_rows)
    if osd_order >= 0:
        decoders.apply_osd(H, syndromes, r.ehat, r.post, r.flags, osd_order, nthreads=1)
    return r


def _bench_leg_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from qldpcsim_amd import decoders
    decoders.decode_batch = _oracle_decode_batch_osd
    out[rank] = {"strong": bench.sim_leg(3, 25, dist, warmup_shots=0, sampler="host"),
                 "weak": bench.sim_leg(3, 12, dist, warmup_shots=0, sampler="host", per_rank=True),
                 "sweep": bench.sim_sweep_leg(4, 6, dist, warmup_shots=0, sampler="host")}
    dist.destroy_process_group()


def test_bench_simulate_legs_two_ranks_gloo():
    """bench.py's end-to-end legs under two gloo ranks (the decode replaced by
    the CPU oracle + host OSD here): configs[3] as a fixed total split over
    the ranks (strong: 25 shots = 13 + 12) and per rank (weak: 2 x 12), and
    configs[4]'s four-point p-sweep through simulate's own p loop. Both ranks
    report the same all-reduced counters, per-rank rates and host cores, the
    OSD shots' host-order share (all of them on this host path), and one curve
    point per p with its own counters."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bench_leg_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    a, b = out[0]["strong"], out[1]["strong"]
    assert a["counters"] == b["counters"] and a["shots"] == b["shots"] == 25 and a["n_ranks"] == 2
    assert a["scaling"] == "strong" and sorted(r["shots"] for r in a["per_rank"]) == [12, 13]
    c = a["counters"]
    assert c["decSuccessExact"] + c["decSuccessDegen"] <= 25 and a["value"] > 0
    assert len(a["per_rank"]) == 2 and all(r["host_cores"] >= 1 and r["shots_per_s"] > 0 for r in a["per_rank"])
    assert a["osd_shots"] == sum(r["osd_shots"] for r in a["per_rank"]) > 0
    assert a["host_order_share"] == 1.0
    w = out[0]["weak"]
    assert w["scaling"] == "weak" and w["shots"] == 24 and [r["shots"] for r in w["per_rank"]] == [12, 12]
    assert w["counters"] == out[1]["weak"]["counters"]
    s0, s1 = out[0]["sweep"], out[1]["sweep"]
    assert s0["p"] == [0.01, 0.02, 0.05, 0.1] and s0["scaling"] == "strong" and s0["n_ranks"] == 2
    assert [pt["p"] for pt in s0["curve"]] == s0["p"] and all(pt["shots"] == 6 for pt in s0["curve"])
    assert [pt["counters"] for pt in s0["curve"]] == [pt["counters"] for pt in s1["curve"]]
    assert all(pt["value"] > 0 and 0.0 <= pt["qBLER"] <= 1.0 for pt in s0["curve"])
    assert s0["elapsed_s"] >= max(pt["elapsed_s"] for pt in s0["curve"])
    # BP never gets OSD from simulate (simulator.py:281-282); iterations are per shot
    assert all(pt["counters"]["Avg_number_of_iterations_X"] >= 1.0 for pt in s0["curve"])
