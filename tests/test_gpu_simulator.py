"""End-to-end simulator on the GPU: counters equal a per-shot restatement of
simulator.py:244-315 driven by the oracle decoders on the same samples; the
CLI runs and prints the reference's table."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("code,decType,sched,osd,p", [
    ("LP04_0", "MS", "F", -1, 0.1),
    ("LP04_0", "MS", "L", 0, 0.12),
    ("LP118_0", "MS", "F", -1, 0.06),
    ("LP04_0", "BP", "L", 4, 0.1),      # BP ignores OSDorder in simulate (simulator.py:281-282)
])
def test_simulate_p_counters_match_oracle_restatement(code, decType, sched, osd, p):
    from oracle import oracle
    from qldpcsim_amd import codes, schedule, simulator
    Hx, Hz = codes.load_code(code)
    shots = 1200
    smp = simulator.sample_channel(Hx, Hz, p, shots, np.random.default_rng(17))
    got = simulator.simulate_p(Hx, Hz, p, shots=shots, decType=decType, decIterations=30,
                               decSchedule=sched, OSDorder=osd, samples=smp, batch_size=1000,
                               verbose=False)
    lx, lz = schedule.select_layers(Hx, Hz, sched)
    sy_z, sy_x, errX, errZ = smp
    outs = []
    for H, layers, syn in ((Hz, lx, sy_z), (Hx, lz, sy_x)):
        lp, lr = schedule.pack_layers(layers, H.shape[0])
        e, it, post, _ = oracle.decode_batch(decType, H, syn, p / 3, 30, lp, lr)
        if decType == "MS" and osd >= 0:
            for k in range(shots):
                if not np.all((H.astype(np.int64) @ e[k]) % 2 == syn[k]):
                    e[k] = oracle.osd_dec(H, e[k].astype(np.int64), syn[k].astype(np.int64),
                                          post[k], osd).astype(np.uint8)
        outs.append((e, it))
    (eX, itX), (eZ, itZ) = outs
    want = dict(DecFailures_X=0, DecFailures_Z=0, decSuccessExact=0, decSuccessDegen=0)
    for k in range(shots):
        if np.array_equal(errX[k], eX[k]) and np.array_equal(errZ[k], eZ[k]):
            want["decSuccessExact"] += 1
        elif ((Hz @ (errX[k].astype(int) ^ eX[k])) == 0).all() and ((Hx @ (errZ[k].astype(int) ^ eZ[k])) == 0).all():
            want["decSuccessDegen"] += 1
        want["DecFailures_X"] += int(not np.array_equal(sy_z[k], (Hz.astype(int) @ eX[k]) % 2))
        want["DecFailures_Z"] += int(not np.array_equal(sy_x[k], (Hx.astype(int) @ eZ[k]) % 2))
    want["Avg_number_of_iterations_X"] = itX.sum() / float(shots)
    want["Avg_number_of_iterations_Z"] = itZ.sum() / float(shots)
    assert got == want


def test_cli_main_prints_reference_table(tmp_path, capsys):
    from qldpcsim_amd import codes, simulator
    Hx, Hz = codes.load_code("LP04_0")
    np.save(tmp_path / "Hx.npy", Hx.astype(np.int64))
    np.save(tmp_path / "Hz.npy", Hz.astype(np.int64))
    simulator.main(["--Hx", str(tmp_path / "Hx.npy"), "--Hz", str(tmp_path / "Hz.npy"),
                    "--p", "0.02", "0.08", "--shots", "2000", "--decType", "MS",
                    "--decIterations", "30", "--decSchedule", "L", "--rngSeed", "5"])
    out = capsys.readouterr().out
    assert "SIMULATION RESULTS" in out and "2.00e-02" in out and "8.00e-02" in out


def test_device_channel_counters_equal_host_counters():
    """DeviceChannel's sampler statistics and its on-device counters equal the
    host restatement (count_outcomes) on the same device-drawn shots."""
    import torch
    from qldpcsim_amd import codes, decoders, simulator
    Hx, Hz = codes.load_code("LP118_0")
    ch = simulator.DeviceChannel(Hx, Hz, torch.device("cuda", 0), 123)
    p = 0.06
    sy_z, sy_x, errXw, errZw = ch.sample(p, 50000)
    errX, errZ = ch.unpack(errXw), ch.unpack(errZw)
    ex = errX.cpu().numpy()
    assert abs(ex.mean() - 2 * p / 3) < 0.002
    np.testing.assert_array_equal(sy_z.cpu().numpy(), (ex.astype(np.int64) @ Hz.T) % 2)
    rX = decoders.decode_batch(Hz, sy_z, p / 3, 30)
    rZ = decoders.decode_batch(Hx, sy_x, p / 3, 30)
    dev = ch.count(sy_z, sy_x, errXw, errZw, rX.ehat, rZ.ehat, rX.iters, rZ.iters)
    host = simulator.count_outcomes(Hx, Hz, sy_z.cpu().numpy(), sy_x.cpu().numpy(), ex,
                                    errZ.cpu().numpy(), rX.ehat.cpu().numpy(), rZ.ehat.cpu().numpy(),
                                    rX.iters.cpu().numpy(), rZ.iters.cpu().numpy())
    assert dev == host


def test_device_sampler_simulate_p_with_osd_agrees_with_host_sampler():
    """Same code/decoder through both samplers: counter rates agree within
    sampling error; OSD on the device path leaves no decoding failure where
    OSD applies (its solve always satisfies a valid syndrome)."""
    from qldpcsim_amd import codes, simulator
    Hx, Hz = codes.load_code("LP04_0")
    kw = dict(shots=20000, decType="MS", decIterations=20, decSchedule="F", rngSeed=3,
              batch_size=8192, verbose=False)
    d = simulator.simulate_p(Hx, Hz, 0.1, OSDorder=0, sampler="device", **kw)
    h = simulator.simulate_p(Hx, Hz, 0.1, OSDorder=0, sampler="host", **kw)
    assert d["DecFailures_X"] == 0 and d["DecFailures_Z"] == 0
    assert h["DecFailures_X"] == 0 and h["DecFailures_Z"] == 0
    for k in ("decSuccessExact",):
        assert abs(d[k] - h[k]) < 5 * np.sqrt(kw["shots"] * 0.25)
    assert abs(d["Avg_number_of_iterations_X"] - h["Avg_number_of_iterations_X"]) < 0.2


@pytest.mark.parametrize("code,p,shot0,B", [
    ("LP118_0", 0.06, 0, 3000),
    ("LP04_0", 0.2, (1 << 32) - 700, 1500),    # the shot counter's high word carries
    ("LP118_2", 0.01, 12345, 1000),
    ("steane", 0.5, 7, 4000),
    ("LP04_0", 1.0, 0, 64),                    # T3 = 2^32: every qubit errs
    ("LP04_0", 0.0, 0, 64),
])
def test_device_sampler_bit_exact_vs_oracle_stream(code, p, shot0, B):
    """qldpc_channel_sample reproduces the oracle's Philox stream bit for bit
    (errors and syndromes), and batching does not change the stream."""
    import torch
    from oracle import oracle
    from qldpcsim_amd import codes, simulator
    Hx, Hz = codes.load_code(code)
    seed = 0x9E3779B97F4A7C15
    ch = simulator.DeviceChannel(Hx, Hz, torch.device("cuda", 0), seed, shot0=shot0)
    a = ch.sample(p, B // 3)
    b = ch.sample(p, B - B // 3)
    got = [torch.cat([x, y]).cpu().numpy() for x, y in zip(a, b)]
    got[2] = ch.unpack(torch.cat([a[2], b[2]])).cpu().numpy()
    got[3] = ch.unpack(torch.cat([a[3], b[3]])).cpu().numpy()
    want = oracle.channel_sample(Hx, Hz, p, seed, shot0, B)
    for g, w, name in zip(got, want, ("sy_z", "sy_x", "errX", "errZ")):
        np.testing.assert_array_equal(g, w, err_msg=name)
    # padding bits of the last word stay zero
    n = Hx.shape[1]
    if n % 64:
        assert int((a[2][:, -1] >> (n % 64)).abs().sum()) == 0


@pytest.mark.parametrize("code,p", [("LP118_0", 0.08), ("LP04_0", 0.15), ("steane", 0.2)])
def test_device_counters_match_reference_loop_with_crafted_estimates(code, p):
    """Counters on estimates built to hit every branch (exact, degenerate-
    style differences on zero-weight columns, failures, iteration sums) equal
    the reference's per-shot loop (simulator.py:291-303)."""
    import torch
    from qldpcsim_amd import codes, simulator
    Hx, Hz = codes.load_code(code)
    dev = torch.device("cuda", 0)
    ch = simulator.DeviceChannel(Hx, Hz, dev, 5)
    B = 2000
    sy_z, sy_x, ewX, ewZ = ch.sample(p, B)
    errX = ch.unpack(ewX).cpu().numpy()
    errZ = ch.unpack(ewZ).cpu().numpy()
    rng = np.random.default_rng(1)
    eX = errX.copy()
    eZ = errZ.copy()
    flip = rng.random((B, eX.shape[1])) < 0.002
    eX ^= flip.astype(np.uint8) * (rng.random(B) < 0.5)[:, None].astype(np.uint8)
    eZ ^= (rng.random((B, eZ.shape[1])) < 0.001).astype(np.uint8)
    itX = rng.integers(1, 60, B).astype(np.int32)
    itZ = rng.integers(1, 60, B).astype(np.int32)
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    got = ch.count(sy_z, sy_x, ewX, ewZ, T(eX), T(eZ), T(itX), T(itZ))
    syz, syx = sy_z.cpu().numpy(), sy_x.cpu().numpy()
    want = dict.fromkeys(simulator.COUNTER_KEYS, 0)
    for k in range(B):
        if np.array_equal(errX[k], eX[k]) and np.array_equal(errZ[k], eZ[k]):
            want["decSuccessExact"] += 1
        elif ((Hz.astype(int) @ (errX[k].astype(int) ^ eX[k])) == 0).all() and \
                ((Hx.astype(int) @ (errZ[k].astype(int) ^ eZ[k])) == 0).all():
            want["decSuccessDegen"] += 1
        want["DecFailures_X"] += int(not np.array_equal(syz[k], (Hz.astype(int) @ eX[k]) % 2))
        want["DecFailures_Z"] += int(not np.array_equal(syx[k], (Hx.astype(int) @ eZ[k]) % 2))
    want["nIterAccX"] = int(itX.sum())
    want["nIterAccZ"] = int(itZ.sum())
    assert got == want
    assert 0 < want["decSuccessExact"] < B and want["DecFailures_X"] > 0


def test_device_counters_degenerate_branch_on_zero_weight_columns():
    """A matrix with an all-zero column: a difference supported there is
    'degenerate' under the reference's integer test (simulator.py:296)."""
    import torch
    from qldpcsim_amd import simulator
    rng = np.random.default_rng(3)
    n = 70
    Hx = (rng.random((12, n)) < 0.2).astype(np.uint8)
    Hz = (rng.random((10, n)) < 0.2).astype(np.uint8)
    Hx[:, 65] = 0
    Hz[:, 65] = 0
    Hz[:, 3] = 0
    dev = torch.device("cuda", 0)
    ch = simulator.DeviceChannel(Hx, Hz, dev, 9)
    B = 300
    sy_z, sy_x, ewX, ewZ = ch.sample(0.1, B)
    errX = ch.unpack(ewX).cpu().numpy()
    errZ = ch.unpack(ewZ).cpu().numpy()
    eX, eZ = errX.copy(), errZ.copy()
    eX[::3, 65] ^= 1
    eX[1::5, 3] ^= 1
    eZ[::7, 65] ^= 1
    eZ[2::11, 3] ^= 1                     # column 3 of Hx is nonzero: not degenerate
    it = np.ones(B, np.int32)
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    got = ch.count(sy_z, sy_x, ewX, ewZ, T(eX), T(eZ), T(it), T(it))
    want = simulator.count_outcomes(Hx, Hz, sy_z.cpu().numpy(), sy_x.cpu().numpy(), errX, errZ,
                                    eX, eZ, it, it)
    assert got == want and want["decSuccessDegen"] > 0


def test_cli_two_ranks_shard_shots(tmp_path):
    """`torchrun -m qldpcsim_amd.simulator` shards the shots over the ranks and
    sums the counters (here 2 ranks share the one GPU over gloo; on the
    8-GPU node one rank per GPU over RCCL)."""
    import json
    import os
    import subprocess
    import sys
    from conftest import ROOT
    from qldpcsim_amd import codes, simulator
    Hx, Hz = codes.load_code("LP04_0")
    np.save(tmp_path / "Hx.npy", Hx.astype(np.int64))
    np.save(tmp_path / "Hz.npy", Hz.astype(np.int64))
    res = tmp_path / "res.json"
    shots = 40001
    env = dict(os.environ, QLDPC_SIM_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29533", "-m", "qldpcsim_amd.simulator",
                        "--Hx", str(tmp_path / "Hx.npy"), "--Hz", str(tmp_path / "Hz.npy"), "--p", "0.08",
                        "--shots", str(shots), "--decIterations", "30", "--rngSeed", "4",
                        "--results", str(res)], cwd=ROOT, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.count("SIMULATION RESULTS") == 1          # rank 0 prints the table
    doc = json.loads(res.read_text())
    assert doc["meta"]["world"] == 2
    two = doc["results"]["0.08"]
    one = simulator.simulate_p(Hx, Hz, 0.08, shots=shots, decIterations=30, rngSeed=4, verbose=False)
    for k in ("decSuccessExact", "DecFailures_X"):
        assert abs(two[k] - one[k]) < 6 * np.sqrt(shots * 0.25) + 5, (k, two[k], one[k])
    assert two["decSuccessExact"] + two["decSuccessDegen"] <= shots
    assert abs(two["Avg_number_of_iterations_X"] - one["Avg_number_of_iterations_X"]) < 0.1


def _oracle_counters(Hx, Hz, sched, decType, osd, p, max_iter, sy_z, sy_x, errX, errZ):
    """The reference's per-shot loop (simulator.py:244-304) on the oracle:
    decode both halves with the cross-wired layers (:278-282), OSD on every
    non-converged MS decode (decoders.py:179-180), then the six counters."""
    from oracle import oracle
    from qldpcsim_amd import schedule
    lx, lz = schedule.select_layers(Hx, Hz, sched)
    outs = []
    for H, layers, syn in ((Hz, lx, sy_z), (Hx, lz, sy_x)):
        lp, lr = schedule.pack_layers(layers, H.shape[0])
        e, it, post, fl = oracle.decode_batch(decType, H, syn, p / 3, max_iter, lp, lr)
        if decType == "MS" and osd >= 0:
            for k in np.flatnonzero((fl & 1) == 0):
                e[k] = oracle.osd_dec(H, e[k].astype(np.int64), syn[k].astype(np.int64), post[k],
                                      osd).astype(np.uint8)
        outs.append((e, it))
    (eX, itX), (eZ, itZ) = outs
    shots = sy_z.shape[0]
    want = dict(DecFailures_X=0, DecFailures_Z=0, decSuccessExact=0, decSuccessDegen=0)
    for k in range(shots):
        if np.array_equal(errX[k], eX[k]) and np.array_equal(errZ[k], eZ[k]):
            want["decSuccessExact"] += 1
        elif ((Hz.astype(int) @ (errX[k].astype(int) ^ eX[k])) == 0).all() and \
                ((Hx.astype(int) @ (errZ[k].astype(int) ^ eZ[k])) == 0).all():
            want["decSuccessDegen"] += 1
        want["DecFailures_X"] += int(not np.array_equal(sy_z[k], (Hz.astype(int) @ eX[k]) % 2))
        want["DecFailures_Z"] += int(not np.array_equal(sy_x[k], (Hx.astype(int) @ eZ[k]) % 2))
    want["Avg_number_of_iterations_X"] = itX.sum() / float(shots)
    want["Avg_number_of_iterations_Z"] = itZ.sum() / float(shots)
    return want, int(((outs[0][1] == max_iter) | (outs[1][1] == max_iter)).sum())


@pytest.mark.parametrize("device_min", ["1", "4096"])   # device reliability order / host order
@pytest.mark.parametrize("decType,osd,p,max_iter,shots,batch", [
    ("MS", 0, 0.1, 50, 330, 100),      # BASELINE configs[3]: LP118_2 MS layered + OSD-0
    ("BP", 4, 0.05, 100, 330, 100),    # configs[4]: LP118_2 BP layered (OSDorder ignored, :281-282)
])
def test_device_pipeline_counters_exact_on_configs_workload(decType, osd, p, max_iter, shots, batch, device_min,
                                                            osdpol):
    """The device simulate_p path (Philox sampler -> decode -> pinned
    posterior staging -> host reliability order -> GPU OSD -> on-device
    counters, two batch slots in flight) over 4 pipelined batches gives
    exactly the counters of the reference's per-shot loop run on the oracle
    with the same shots."""
    import torch
    from qldpcsim_amd import codes, simulator
    osdpol(device_min=int(device_min))
    Hx, Hz = codes.load_code("LP118_2")
    seed = 11
    got = simulator.simulate_p(Hx, Hz, p, shots=shots, decType=decType, decIterations=max_iter,
                               decSchedule="L", OSDorder=osd, rngSeed=seed, batch_size=batch,
                               sampler="device", verbose=False)
    # the same shots: simulate_p's stream for (rngSeed, rank 0), shot 0 on
    key = np.random.SeedSequence([seed, 0]).generate_state(1, np.uint64)[0]
    ch = simulator.DeviceChannel(Hx, Hz, torch.device("cuda", 0), key)
    sy_z, sy_x, ewX, ewZ = ch.sample(p, shots)
    errX, errZ = ch.unpack(ewX).cpu().numpy(), ch.unpack(ewZ).cpu().numpy()
    want, capped = _oracle_counters(Hx, Hz, "L", decType, osd, p, max_iter, sy_z.cpu().numpy(),
                                    sy_x.cpu().numpy(), errX, errZ)
    assert got == want
    if decType == "MS":
        assert capped > 50                  # OSD ran on many shots of every batch


def test_simulator_refuses_more_ranks_than_gpus_over_rccl(monkeypatch):
    """Under RCCL one rank per GPU: a LOCAL_RANK past the visible devices is a
    launch error (raised before the process group forms), as bench.py's; the
    gloo rehearsal switch still lets ranks share a device."""
    import torch
    from qldpcsim_amd import simulator
    n = torch.cuda.device_count()
    monkeypatch.setenv("WORLD_SIZE", str(n + 1))
    monkeypatch.setenv("RANK", str(n))
    monkeypatch.setenv("LOCAL_RANK", str(n))
    monkeypatch.delenv("QLDPC_SIM_BACKEND", raising=False)
    with pytest.raises(RuntimeError, match="HIP device"):
        simulator._init_dist_from_env()


@pytest.mark.parametrize("device_min", ["1", "4096"])   # device reliability order / host order
def test_two_ranks_configs3_pipeline_counters_exact(tmp_path, device_min):
    """configs[3]'s pipeline (LP118_2 MS layered + OSD-0, p = 0.1, 50
    iterations) under `torchrun --nproc-per-node 2` (gloo, both ranks on the
    one GPU, 2 batches each): the all-reduced counters equal EXACTLY the sum
    of the reference's per-shot loop run on the oracle over each rank's own
    shots — rank r's contiguous share, drawn from its Philox key (rngSeed, r)
    — i.e. the sharding adds, drops and repeats no shot (simulator.py:244-315)."""
    import json
    import os
    import subprocess
    import sys
    import torch
    from conftest import ROOT
    from qldpcsim_amd import codes, simulator
    Hx, Hz = codes.load_code("LP118_2")
    np.save(tmp_path / "Hx.npy", Hx.astype(np.int64))
    np.save(tmp_path / "Hz.npy", Hz.astype(np.int64))
    res = tmp_path / "res.json"
    shots, seed, p, it = 241, 13, 0.1, 50
    env = dict(os.environ, QLDPC_SIM_BACKEND="gloo", QLDPC_OSD_DEVICE_MIN=device_min)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29537", "-m", "qldpcsim_amd.simulator",
                        "--Hx", str(tmp_path / "Hx.npy"), "--Hz", str(tmp_path / "Hz.npy"), "--p", str(p),
                        "--shots", str(shots), "--decIterations", str(it), "--decSchedule", "L",
                        "--OSDorder", "0", "--rngSeed", str(seed), "--batch", "64", "--results", str(res)],
                       cwd=ROOT, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads(res.read_text())["results"][str(p)]
    want = {k: 0 for k in ("DecFailures_X", "DecFailures_Z", "decSuccessExact", "decSuccessDegen")}
    its = [0.0, 0.0]
    capped = 0
    for rank in range(2):
        my = shots // 2 + (1 if rank < shots % 2 else 0)
        key = np.random.SeedSequence([seed, rank]).generate_state(1, np.uint64)[0]
        ch = simulator.DeviceChannel(Hx, Hz, torch.device("cuda", 0), key)
        sy_z, sy_x, ewX, ewZ = ch.sample(p, my)
        w, c = _oracle_counters(Hx, Hz, "L", "MS", 0, p, it, sy_z.cpu().numpy(), sy_x.cpu().numpy(),
                                ch.unpack(ewX).cpu().numpy(), ch.unpack(ewZ).cpu().numpy())
        for k in want:
            want[k] += w[k]
        its[0] += w["Avg_number_of_iterations_X"] * my
        its[1] += w["Avg_number_of_iterations_Z"] * my
        capped += c
    for k in want:
        assert got[k] == want[k], (k, got[k], want[k])
    assert abs(got["Avg_number_of_iterations_X"] - its[0] / shots) < 1e-9
    assert abs(got["Avg_number_of_iterations_Z"] - its[1] / shots) < 1e-9
    assert capped > 50                                      # OSD ran on many shots of both ranks


def test_device_pipeline_counters_independent_of_batching():
    """The device pipeline's tail batches are halved when OSD is a large
    share of a batch (simulate_p): shots keep the sampler's indices, so the
    counters of a sweep point are the same whatever the batch sequence —
    here one batch, full batches, and full batches plus the tapered tail
    (LP04_0 MS-L + OSD-0 at p = 0.12: most half-shots need OSD)."""
    from qldpcsim_amd import codes, simulator
    Hx, Hz = codes.load_code("LP04_0")
    kw = dict(shots=3000, decType="MS", decIterations=30, decSchedule="L", OSDorder=0, rngSeed=5,
              verbose=False, sampler="device")
    runs = [simulator.simulate_p(Hx, Hz, 0.12, batch_size=b, **kw) for b in (3000, 1000, 512)]
    assert runs[0] == runs[1] == runs[2], runs
