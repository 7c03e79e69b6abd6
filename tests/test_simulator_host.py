"""Host logic of the drop-in simulator: matrix loading, layer construction and
cross-wiring, outcome counting, the channel sampler and the results table."""
import numpy as np
import pytest

from qldpcsim_amd import codes, schedule
from qldpcsim_amd.simulator import count_outcomes, format_results, load_matrix, sample_channel


def _layerize_literal(H, serial=False):
    # simulator.py:212-224, restated independently
    out, m, up, dn = [], H.shape[0], 1, 0
    while up <= m:
        if H[dn:up].sum(axis=0).max() > 1 or (serial and up > dn + 1):
            out.append(list(range(dn, up - 1)))
            dn = up - 1
        else:
            up += 1
    out.append(list(range(dn, up - 1)))
    return out


@pytest.mark.parametrize("name,nx,nz", [("LP118_0", 13, 11), ("LP118_2", 13, 11), ("LP04_0", 10, 9)])
def test_layer_counts_match_survey(name, nx, nz):
    Hx, Hz = codes.load_code(name)
    lx, lz = schedule.select_layers(Hx, Hz, "L")
    assert (len(lx), len(lz)) == (nx, nz)
    for H, ls in ((Hx, lx), (Hz, lz)):
        assert [list(l) for l in ls] == _layerize_literal(H)
        for l in ls:                                    # column-disjoint on the matrix they came from
            assert H[l].sum(axis=0).max() <= 1


def test_layers_equal_reference_layerize():
    """schedule.select_layers equals the layers the reference's own layerize /
    schedule selection (simulator.py:212-236, executed by
    tests/golden/gen_golden_layers.py) builds for every bundled code, L and S,
    cross-wiring included: layersX (from Hx) decodes Hz, layersZ decodes Hx."""
    import json
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", "schedules", "layers.npz")
    with np.load(path, allow_pickle=False) as z:
        keys = json.loads(bytes(z["index_json"]).decode())["keys"]
        assert len(keys) == 4 * len(codes.available())
        for key in keys:
            name, sched, half = key.split("__")
            Hx, Hz = codes.load_code(name)
            lx, lz = schedule.select_layers(Hx, Hz, sched)
            # (packed against the matrix the layers came from: a code whose Hx and Hz
            # differ in rows would make pack_layers raise the reference's IndexError)
            ptr, rows = schedule.pack_layers(lx if half == "X" else lz, (Hx if half == "X" else Hz).shape[0])
            assert np.array_equal(ptr, z[key + "__ptr"]) and np.array_equal(rows, z[key + "__rows"]), key


def test_serial_and_flooding_layers():
    Hx, Hz = codes.load_code("LP04_0")
    sx, sz = schedule.select_layers(Hx, Hz, "S")
    assert [list(l) for l in sx] == [[i] for i in range(Hx.shape[0])]
    fx, fz = schedule.select_layers(Hx, Hz, "F")
    assert len(fx) == 1 and list(fx[0]) == list(range(Hx.shape[0]))
    with pytest.raises(ValueError, match="Unrecognized decoder scheduling option"):
        schedule.select_layers(Hx, Hz, "Q")


def test_pack_layers():
    ptr, rows = schedule.pack_layers([np.array([0, 2]), np.array([1])], 3)
    assert ptr.tolist() == [0, 2, 3] and rows.tolist() == [0, 2, 1]
    with pytest.raises(IndexError):
        schedule.pack_layers([np.array([5])], 3)
    p2, r2 = schedule.pack_layers(None, 4)
    assert p2.tolist() == [0, 4] and r2.tolist() == [0, 1, 2, 3]


def test_load_matrix_npy_and_text(tmp_path):
    M = np.array([[1, 0, 3], [2, 1, 1]])
    np.save(tmp_path / "m.npy", M)
    (tmp_path / "m.txt").write_text("1 0 3\n\n2 1 1\n")
    for p in ("m.npy", "m.txt"):
        L = load_matrix(str(tmp_path / p))
        assert L.dtype == np.int8
        np.testing.assert_array_equal(L, M % 2)


def _count_literal(Hx, Hz, sy_z, sy_x, errX, errZ, eX, eZ, itX, itZ):
    # simulator.py:291-303, one shot at a time
    c = dict(DecFailures_X=0, DecFailures_Z=0, decSuccessExact=0, decSuccessDegen=0,
             nIterAccX=0, nIterAccZ=0)
    for k in range(len(itX)):
        c["nIterAccX"] += int(itX[k])
        c["nIterAccZ"] += int(itZ[k])
        ex, ez = errX[k].astype(int), errZ[k].astype(int)
        dx, dz = eX[k].astype(np.int8), eZ[k].astype(np.int8)
        if np.array_equal(ex, dx) and np.array_equal(ez, dz):
            c["decSuccessExact"] += 1
        elif ((Hz @ (ex ^ dx)) == 0).all() and ((Hx @ (ez ^ dz)) == 0).all():
            c["decSuccessDegen"] += 1
        if not np.array_equal(sy_z[k].astype(int), (Hz.dot(dx)) % 2):
            c["DecFailures_X"] += 1
        if not np.array_equal(sy_x[k].astype(int), (Hx.dot(dz)) % 2):
            c["DecFailures_Z"] += 1
    return c


def test_count_outcomes_matches_per_shot_restatement():
    rng = np.random.default_rng(3)
    Hx, Hz = codes.load_code("LP04_0")
    B = 300
    sy_z, sy_x, errX, errZ = sample_channel(Hx, Hz, 0.08, B, rng)
    # estimates: exact for some shots, syndrome-equivalent for others, wrong for the rest
    eX, eZ = errX.copy(), errZ.copy()
    flip = rng.random(B) < 0.3
    eX[flip, rng.integers(0, Hx.shape[1], flip.sum())] ^= 1
    eZ[rng.random(B) < 0.2, 0] ^= 1
    Hs = Hx.astype(np.int64)                      # a stabilizer of the X-check space
    sel = rng.random(B) < 0.1
    eZ[sel] ^= Hs[0].astype(np.uint8)
    itX = rng.integers(1, 50, B)
    itZ = rng.integers(1, 50, B)
    got = count_outcomes(Hx, Hz, sy_z, sy_x, errX, errZ, eX, eZ, itX, itZ)
    assert got == _count_literal(Hx, Hz, sy_z, sy_x, errX, errZ, eX, eZ, itX, itZ)


def test_channel_sampler_statistics_and_syndromes():
    rng = np.random.default_rng(11)
    Hx, Hz = codes.load_code("LP118_0")
    p = 0.06
    sy_z, sy_x, errX, errZ = sample_channel(Hx, Hz, p, 20000, rng)
    # X flip marginal = P(X)+P(Y) = 2p/3
    assert abs(errX.mean() - 2 * p / 3) < 0.002 and abs(errZ.mean() - 2 * p / 3) < 0.002
    assert abs((errX & errZ).mean() - p / 3) < 0.002             # Y errors
    np.testing.assert_array_equal(sy_z, (errX.astype(np.int64) @ Hz.T) % 2)
    np.testing.assert_array_equal(sy_x, (errZ.astype(np.int64) @ Hx.T) % 2)


def test_results_table_format():
    r = {"decSuccessExact": 990, "decSuccessDegen": 0, "DecFailures_X": 3, "DecFailures_Z": 4,
         "Avg_number_of_iterations_X": 1.25, "Avg_number_of_iterations_Z": 1.5}
    txt = format_results([0.01], [r], 1000)
    assert "SIMULATION RESULTS" in txt
    assert "  1.00e-02  " in txt and "1.00e-02" in txt and "    3,    4" in txt and " 1.25,  1.50" in txt


def test_oracle_philox_known_answer_vectors():
    """The oracle's Philox4x32-10 block function reproduces the published
    known-answer vectors (Random123 kat_vectors, philox4x32_10)."""
    import ctypes
    from oracle import oracle
    L = oracle.lib()
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in kat:
        c = np.array(ctr, np.uint32)
        L.oracle_philox4x32_10(c.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(key[0]),
                               ctypes.c_uint32(key[1]))
        assert tuple(int(x) for x in c) == want


def test_oracle_channel_stream_statistics_and_thresholds():
    """The sampler stream restatement: X/Y/Z each p/3 per qubit (simulator.py:107),
    syndromes H·e mod 2, thresholds match the C ABI's."""
    import ctypes
    from oracle import oracle
    from qldpcsim_amd import _lib, codes
    for p in (0.0, 0.01, 0.3, 1.0):
        t = [ctypes.c_uint64() for _ in range(3)]
        _lib.check(_lib.lib.qldpc_channel_thresholds(p, *(ctypes.byref(x) for x in t)))
        assert tuple(x.value for x in t) == oracle.channel_thresholds(p)
    with pytest.raises(ValueError):
        _lib.check(_lib.lib.qldpc_channel_thresholds(1.5, None, None, None))
    Hx, Hz = codes.load_code("LP04_0")
    p = 0.09
    sz, sx, ex, ez = oracle.channel_sample(Hx, Hz, p, 77, 0, 6000)
    N = ex.size
    y = (ex & ez).mean()
    assert abs(y - p / 3) < 5 * np.sqrt(p / 3 / N)
    assert abs((ex & (1 - ez)).mean() - p / 3) < 5 * np.sqrt(p / 3 / N)
    assert abs((ez & (1 - ex)).mean() - p / 3) < 5 * np.sqrt(p / 3 / N)
    np.testing.assert_array_equal(sz, (ex.astype(np.int64) @ Hz.T) % 2)
    np.testing.assert_array_equal(sx, (ez.astype(np.int64) @ Hx.T) % 2)
    # the stream is a function of (seed, shot): an offset window matches
    w = oracle.channel_sample(Hx, Hz, p, 77, 1000, 50)
    np.testing.assert_array_equal(w[2], ex[1000:1050])


def test_resumable_results_file(tmp_path, monkeypatch):
    """simulate(resultsFile=...) writes each p-point as it finishes and a rerun
    skips the points already there; a file from another run is refused."""
    from qldpcsim_amd import simulator
    calls = []

    def fake_simulate_p(Hx, Hz, p, **kw):
        calls.append(p)
        return {"DecFailures_X": 1, "DecFailures_Z": 2, "decSuccessExact": 90, "decSuccessDegen": 0,
                "Avg_number_of_iterations_X": 1.5, "Avg_number_of_iterations_Z": p}

    monkeypatch.setattr(simulator, "simulate_p", fake_simulate_p)
    Hx, Hz = codes.load_code("steane")
    np.save(tmp_path / "Hx.npy", Hx)
    np.save(tmp_path / "Hz.npy", Hz)
    f = str(tmp_path / "res.json")
    kw = dict(shots=100, rngSeed=1, verbose=False, return_results=True, resultsFile=f)
    a = simulator.simulate(str(tmp_path / "Hx.npy"), str(tmp_path / "Hz.npy"), [0.01, 0.02], **kw)
    assert calls == [0.01, 0.02]
    b = simulator.simulate(str(tmp_path / "Hx.npy"), str(tmp_path / "Hz.npy"), [0.01, 0.02, 0.05], **kw)
    assert calls == [0.01, 0.02, 0.05] and b[:2] == a
    with pytest.raises(ValueError):
        simulator.simulate(str(tmp_path / "Hx.npy"), str(tmp_path / "Hz.npy"), [0.01],
                           **{**kw, "shots": 200})


def test_samples_with_device_sampler_is_rejected():
    from qldpcsim_amd import codes, simulator
    Hx, Hz = codes.load_code("steane")
    smp = simulator.sample_channel(Hx, Hz, 0.1, 4, np.random.default_rng(0))
    with pytest.raises(ValueError):
        simulator.simulate_p(Hx, Hz, 0.1, shots=4, samples=smp, sampler="device", verbose=False)
    with pytest.raises(ValueError):
        simulator.simulate_p(Hx, Hz, 0.1, shots=4, samples=smp, sampler="gpu", verbose=False)


def test_results_file_records_the_sampler(tmp_path):
    """A resumed sweep must not mix host-stream and device-stream p-points:
    the resolved sampler is part of the results file's run parameters."""
    import json
    from qldpcsim_amd import simulator
    path = str(tmp_path / "res.json")
    meta = {"Hx": "a", "Hz": "b", "shots": 10, "decType": "MS", "decIterations": 5, "decSchedule": "F",
            "OSDorder": -1, "rngSeed": 1, "world": 1, "sampler": "device"}
    simulator._save_results(path, meta, {0.1: {"decSuccessExact": 3}})
    assert simulator._load_results(path, meta) == {0.1: {"decSuccessExact": 3}}
    with pytest.raises(ValueError):
        simulator._load_results(path, dict(meta, sampler="host"))
    assert json.load(open(path))["meta"]["sampler"] == "device"


def test_large_codes_use_the_host_sampler():
    from qldpcsim_amd import simulator
    assert simulator._channel_ok(np.zeros((3, 4096)), np.zeros((3, 4096)))
    assert not simulator._channel_ok(np.zeros((3, 4097)), np.zeros((3, 4097)))


def test_rank_cores_shared_unless_declared_own(monkeypatch):
    """hostcores.rank_cores divides the process budget among the node's ranks
    (LOCAL_WORLD_SIZE) — also when the affinity mask is smaller than the
    machine, since a container cpuset / Slurm allocation / `taskset` on the
    launcher gives every rank the same mask (8 ranks on a 16-CPU cpuset: 2
    threads each, not 16) — and keeps a rank's whole set only when the
    launcher declares it the rank's own (QLDPC_RANK_CPUSET=own)."""
    import os
    from qldpcsim_amd import hostcores
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    monkeypatch.delenv("QLDPC_RANK_CPUSET", raising=False)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setattr(os, "cpu_count", lambda: 128)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(16)))         # a shared 16-CPU cpuset
    monkeypatch.setattr(hostcores, "process_cores", lambda: (16, "sched_getaffinity"))
    assert hostcores.rank_cores() == 2
    monkeypatch.setenv("QLDPC_RANK_CPUSET", "own")                                    # one CPU set per rank
    assert hostcores.rank_cores() == 16
    monkeypatch.delenv("QLDPC_RANK_CPUSET")
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(128)))        # whole machine, shared
    monkeypatch.setattr(hostcores, "process_cores", lambda: (128, "sched_getaffinity"))
    assert hostcores.rank_cores() == 16 and hostcores.rank_cores(cap=64) == 16
    monkeypatch.setattr(hostcores, "process_cores", lambda: (64, "cgroup cpu.max"))
    assert hostcores.rank_cores() == 8
