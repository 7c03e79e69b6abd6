"""Throughput of the BASELINE.json configs (and variants) on one GPU.

Each line: decode kernel time per launch and shots/s for one (code, algo,
schedule, syndrome source) point, with syndromes resident on the device.
Channel syndromes use the per-qubit Pauli sampler.
usage: python tools/bench_configs.py [--quick]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import _lib, codes, decoders, schedule  # noqa: E402


def channel(Hx, Hz, p, B, gen):
    n = Hx.shape[1]
    u = torch.rand((B, n), device="cuda", generator=gen)
    X = u < p / 3
    Y = (u >= p / 3) & (u < 2 * p / 3)
    Z = (u >= 2 * p / 3) & (u < p)
    ex, ez = (X | Y).half(), (Z | Y).half()
    sz = (ex @ torch.as_tensor(Hz.T, dtype=torch.half, device="cuda")).remainder_(2).to(torch.uint8)
    sx = (ez @ torch.as_tensor(Hx.T, dtype=torch.half, device="cuda")).remainder_(2).to(torch.uint8)
    return sz.contiguous(), sx.contiguous()


def run(code, algo, sched, p, max_iter, B, reps=2):
    Hx, Hz = codes.load_code(code)
    lx, lz = schedule.select_layers(Hx, Hz, sched)
    gen = torch.Generator(device="cuda").manual_seed(7)
    if p is None:
        sz = torch.randint(0, 2, (B, Hz.shape[0]), dtype=torch.uint8, device="cuda", generator=gen)
        sx = torch.randint(0, 2, (B, Hx.shape[0]), dtype=torch.uint8, device="cuda", generator=gen)
        prior = 0.05 / 3
    else:
        sz, sx = channel(Hx, Hz, p, B, gen)
        prior = p / 3
    halves = ((Hz, lx, sz), (Hx, lz, sx))
    packed = [schedule.pack_layers(l, H.shape[0]) for H, l, _ in halves]
    for (H, _, s), (lp, lr) in zip(halves, packed):        # warm-up / graph upload
        decoders.decode_batch(H, s[:1024], prior, max_iter, algo=algo, layer_ptr=lp, layer_rows=lr)
    torch.cuda.synchronize()
    _lib.timing_enable(True)
    _lib.timing_reset()
    its = 0
    t0 = time.perf_counter()
    for _ in range(reps):
        for (H, _, s), (lp, lr) in zip(halves, packed):
            r = decoders.decode_batch(H, s, prior, max_iter, algo=algo, layer_ptr=lp, layer_rows=lr)
            its += int(r.iters.sum().item())
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms, nl = _lib.timing_read()
    _lib.timing_enable(False)
    return {"code": code, "algo": algo, "sched": sched, "p": p, "max_iter": max_iter, "batch": B,
            "kernel_ms_per_launch": ms / nl, "shots_per_s_kernel": reps * B / (ms / 1e3),
            "shots_per_s_wall": reps * B / wall, "avg_iters": its / (2 * reps * B)}


def run_hbm(n, dv, dc, algo, p, max_iter, B, force_code=None):
    """The HBM-resident kernel: a synthetic (dv, dc)-regular code of n
    variables (or a bundled code with the force_hbm option), one launch per half;
    achieved GB/s under SURVEY.md 8(d)'s streaming model, w(3E + 2n) bytes
    per executed half-shot iteration (w = 4 MS / 8 BP), against 8 TB/s."""
    if force_code:
        _lib.set_option("force_hbm", 1)
        Hx, Hz = codes.load_code(force_code)
        H = Hz
    else:
        rng = np.random.default_rng(1)
        m = n * dv // dc
        H = np.zeros((m, n), np.uint8)
        H[rng.permutation(np.repeat(np.arange(m), dc)), np.repeat(np.arange(n), dv)] = 1
    m, n = H.shape
    E = int(H.sum())
    gen = torch.Generator(device="cuda").manual_seed(3)
    if p is None:
        s = torch.randint(0, 2, (B, m), dtype=torch.uint8, device="cuda", generator=gen)
        prior = 0.05 / 3
    else:
        e = (torch.rand((B, n), device="cuda", generator=gen) < p).half()
        s = (e @ torch.as_tensor(H.T, dtype=torch.half, device="cuda")).remainder_(2).to(torch.uint8)
        prior = p / 3
    lp, lr = np.array([0, m], np.int32), np.arange(m, dtype=np.int32)
    name = _lib.kernel_name(H, lp, lr, algo)
    decoders.decode_batch(H, s[:256], prior, max_iter, algo=algo, layer_ptr=lp, layer_rows=lr)
    torch.cuda.synchronize()
    _lib.timing_enable(True)
    _lib.timing_reset()
    r = decoders.decode_batch(H, s, prior, max_iter, algo=algo, layer_ptr=lp, layer_rows=lr)
    its = int(r.iters.sum().item())
    ms, nl = _lib.timing_read()
    _lib.timing_enable(False)
    _lib.set_option("force_hbm", 0)
    w = 4 if algo == "MS" else 8
    byts = its * (w * (3 * E + 2 * n)) + B * (m + n + 4)
    return {"hbm_kernel": name, "code": force_code or f"regular({dv},{dc}) n={n}", "m": m, "n": n, "E": E,
            "algo": algo, "p": p, "max_iter": max_iter, "batch": B, "kernel_ms": ms / nl,
            "half_shots_per_s": B / (ms / 1e3), "avg_iters": its / B,
            "algorithmic_gbs": byts / (ms / 1e3) / 1e9, "hbm_frac": byts / (ms / 1e3) / 1e9 / 8000.0}


def run_osd(code, count, order=0):
    """GPU OSD throughput on random posteriors / arbitrary syndromes."""
    Hx, Hz = codes.load_code(code)
    H = Hz
    rng = np.random.default_rng(1)
    post = rng.normal(0, 3, (count, H.shape[1]))
    t0 = time.perf_counter()
    perms = torch.as_tensor(decoders.osd_perms(post), device="cuda")
    t_perm = time.perf_counter() - t0
    syn = torch.randint(0, 2, (count, H.shape[0]), dtype=torch.uint8, device="cuda")
    e = torch.as_tensor((post < 0).astype(np.uint8), device="cuda")
    st = torch.empty(count, dtype=torch.int32, device="cuda")
    code_h = _lib.code_for(H, 0)
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _lib.check(_lib.lib.qldpc_osd_device(code_h.handle, count, syn.data_ptr(), perms.data_ptr(), order,
                                             e.data_ptr(), st.data_ptr(), None))
        torch.cuda.synchronize()
        t_gpu = time.perf_counter() - t0
    return {"osd_code": code, "count": count, "order": order, "gpu_osd_per_s": count / t_gpu,
            "host_perm_per_s": count / t_perm}


def main():
    quick = "--quick" in sys.argv
    S = 1 << (16 if quick else 18)
    pts = [
        ("LP118_0", "MS", "F", None, 50, S * 4),
        ("LP118_0", "MS", "F", 0.01, 50, S * 4),
        ("LP118_0", "MS", "F", 0.05, 50, S * 4),
        ("LP04_0", "MS", "F", 0.05, 50, S * 4),             # configs[1]
        ("LP118_0", "MS", "L", None, 50, S),
        ("LP118_0", "BP", "F", 0.05, 100, S),                # configs[2]
        ("LP118_0", "BP", "L", 0.05, 100, S),
        ("LP118_0", "BP", "F", None, 100, S // 4),
        ("LP118_2", "MS", "L", 0.05, 50, S),                 # configs[3] (decoder part)
        ("LP118_2", "MS", "F", None, 50, S),
        ("LP118_2", "BP", "L", 0.05, 100, S // 2),           # configs[4] (decoder part)
    ]
    if "--hbm-large" in sys.argv:
        # batches that fill the chip: the kernel keeps min(batch, 16 waves per
        # CU, 64 GB of state) slots resident (capi.cpp decode_hbm)
        for pt in [(16384, 3, 6, "MS", None, 20, 196608), (16384, 3, 6, "MS", 0.02, 50, 262144),
                   (16384, 3, 6, "BP", None, 10, 98304)]:
            print(json.dumps(run_hbm(*pt)), flush=True)
        return
    if "--hbm" in sys.argv:
        for pt in [(16384, 3, 6, "MS", None, 50, 16384), (16384, 3, 6, "MS", 0.02, 50, 65536),
                   (16384, 3, 6, "BP", None, 20, 8192), (None, None, None, "MS", None, 50, 65536, "LP118_0")]:
            print(json.dumps(run_hbm(*pt)), flush=True)
        return
    if "--osd" in sys.argv:
        for c in ("LP04_0", "LP118_0", "LP118_2"):
            print(json.dumps(run_osd(c, 8192)), flush=True)
        return
    for pt in pts:
        print(json.dumps(run(*pt)), flush=True)


if __name__ == "__main__":
    main()
