"""Generate golden decoder vectors from the UNMODIFIED reference decoders.

Build container only: imports /root/reference/qLDPCsim/decoders.py through a
stub package (the real qLDPCsim/__init__.py needs the absent `tomlkit`;
SURVEY.md §8c / App. B). Nothing here runs on the GPU box; the outputs are
committed as data fixtures (`tests/golden/*.npz`): inputs (syndromes, layers,
p, max_iter) and the reference's outputs (ê, iteration count, and the final
posterior LLRs captured with a sys.settrace return hook on MS_decoder /
BP_decoder — decoders.py:173 `posteriorLLRs`, :276 `L_post`).

Usage:  python tests/golden/gen_golden.py            (≈ a few minutes, 8 procs)
"""
import importlib
import json
import os
import sys
import types
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from qldpcsim_amd import codes, schedule  # noqa: E402  (host logic only: data + layerize)

REF = "/root/reference/qLDPCsim"
_dec = None


def ref_decoders():
    global _dec
    if _dec is None:
        sys.dont_write_bytecode = True
        pkg = types.ModuleType("qLDPCsim")
        pkg.__path__ = [REF]
        sys.modules["qLDPCsim"] = pkg
        _dec = importlib.import_module("qLDPCsim.decoders")
    return _dec


def run_capture(fn, capture_name, *args, **kw):
    """Call fn, capturing local `capture_name` of the decoder frame at return."""
    box = {}
    target = fn.__code__

    def tracer(frame, event, arg):
        if frame.f_code is target:
            def local(fr, ev, a):
                if ev == "return" and capture_name in fr.f_locals:
                    box["v"] = np.array(fr.f_locals[capture_name], dtype=np.float64, copy=True)
                return local
            return local
        return None

    sys.settrace(tracer)
    try:
        out = fn(*args, **kw)
    finally:
        sys.settrace(None)
    return out, box.get("v")


def channel_syndromes(Hx, Hz, p, shots, rng):
    """Per-qubit Pauli draw (X, Y, Z each p/3); SURVEY.md App. A.5."""
    n = Hx.shape[1]
    u = rng.random((shots, n))
    X = u < p / 3
    Y = (u >= p / 3) & (u < 2 * p / 3)
    Z = (u >= 2 * p / 3) & (u < p)
    errX = (X | Y).astype(np.int64)
    errZ = (Z | Y).astype(np.int64)
    sy_z = (errX @ Hz.T.astype(np.int64)) % 2
    sy_x = (errZ @ Hx.T.astype(np.int64)) % 2
    return sy_z, sy_x, errX, errZ


def half_inputs(code, half, sched):
    Hx, Hz = codes.load_code(code)
    layersX, layersZ = schedule.select_layers(Hx, Hz, sched)
    if half == "X":
        return Hz, layersX
    return Hx, layersZ


def run_case(case):
    dec = ref_decoders()
    H, layers = half_inputs(case["code"], case["half"], case["sched"])
    if max(int(np.max(l)) if len(l) else -1 for l in layers) >= H.shape[0]:
        # cross-wired layers index rows H does not have (e.g. shor, m_x != m_z):
        # the reference raises IndexError (decoders.py:156 / :250); record that.
        s = np.ones(H.shape[0], dtype=int)
        fn = dec.MS_decoder if case["algo"] == "MS" else dec.BP_decoder
        try:
            fn(H, s, p=case["p_phys"] / 3, max_iter=1, layers=layers)
        except IndexError:
            case = dict(case, raises="IndexError")
            return case, {}
        return dict(case, raises="none-for-all-ones"), {}
    Hx, Hz = codes.load_code(case["code"])
    rng = np.random.default_rng(case["seed"])
    K = case["shots"]
    if case["kind"] == "channel":
        sy_z, sy_x, _, _ = channel_syndromes(Hx, Hz, case["p_phys"], K, rng)
        syn = sy_z if case["half"] == "X" else sy_x
    else:
        syn = rng.integers(0, 2, size=(K, H.shape[0]), dtype=np.int64)
    prior = case["p_phys"] / 3.0
    m, n = H.shape
    ehat = np.zeros((K, n), np.uint8)
    iters = np.zeros(K, np.int32)
    post = np.zeros((K, n), np.float64)
    for k in range(K):
        s = syn[k].astype(int)
        if case["algo"] == "MS":
            (e, it), pst = run_capture(dec.MS_decoder, "posteriorLLRs", H, s, p=prior,
                                       max_iter=case["max_iter"], layers=layers,
                                       OSDorder=case["osd"])
        else:
            (e, it), pst = run_capture(dec.BP_decoder, "L_post", H, s, p=prior,
                                       max_iter=case["max_iter"], layers=layers,
                                       OSDorder=case["osd"])
        ehat[k] = np.asarray(e).astype(np.uint8)
        iters[k] = it
        post[k] = pst
    lp, lr = schedule.pack_layers(layers, m)
    return case, dict(syn=syn.astype(np.uint8), ehat=ehat, iters=iters, post=post,
                      layer_ptr=lp, layer_rows=lr)


def build_cases():
    cases = []
    seed = 20251226

    def add(**kw):
        nonlocal seed
        seed += 1
        kw.setdefault("osd", -1)
        kw["seed"] = seed
        cases.append(kw)

    # --- Min-Sum -------------------------------------------------------------
    small = ["steane", "LP04_0", "shor", "bicycle"]
    for code in small + ["LP118_0", "LP118_2"]:
        for half in ("X", "Z"):
            for sched in ("F", "L", "S"):
                big = code in ("LP118_0", "LP118_2")
                if sched == "S" and code == "LP118_2":
                    continue
                K = 6 if big else 12
                if sched == "S" and big:
                    K = 3
                for p in (0.02, 0.08, 0.15):
                    add(algo="MS", code=code, half=half, sched=sched, kind="channel",
                        p_phys=p, shots=K, max_iter=3 if (sched == "S" and big) else 50)
                for mi in (1, 2, 7):
                    add(algo="MS", code=code, half=half, sched=sched, kind="random",
                        p_phys=0.05, shots=2 if big else 4, max_iter=mi if not (sched == "S" and big) else min(mi, 2))
    # --- BP ------------------------------------------------------------------
    for code in ["steane", "LP04_0", "shor", "bicycle", "LP118_0"]:
        for half in ("X", "Z"):
            for sched in ("F", "L", "S"):
                big = code == "LP118_0"
                if sched == "S" and code in ("LP118_0", "bicycle"):
                    continue
                K = 3 if big else 8
                for p in (0.02, 0.08):
                    add(algo="BP", code=code, half=half, sched=sched, kind="channel",
                        p_phys=p, shots=K, max_iter=20 if big else 30)
                for mi in (1, 3):
                    add(algo="BP", code=code, half=half, sched=sched, kind="random",
                        p_phys=0.05, shots=2, max_iter=mi)
    # --- OSD post-decoding (decoders.py:179-180, :287-288) ------------------
    for order in (0, 1, 2, 4):
        add(algo="MS", code="LP04_0", half="X", sched="F", kind="random", p_phys=0.05,
            shots=3, max_iter=5, osd=order)
        add(algo="MS", code="steane", half="Z", sched="L", kind="random", p_phys=0.1,
            shots=4, max_iter=3, osd=order)
    add(algo="MS", code="LP04_0", half="Z", sched="L", kind="channel", p_phys=0.15,
        shots=6, max_iter=4, osd=0)
    add(algo="MS", code="LP118_0", half="X", sched="F", kind="random", p_phys=0.05,
        shots=1, max_iter=3, osd=0)
    add(algo="MS", code="LP118_0", half="Z", sched="F", kind="random", p_phys=0.05,
        shots=1, max_iter=3, osd=1)
    add(algo="BP", code="LP04_0", half="X", sched="F", kind="random", p_phys=0.05,
        shots=2, max_iter=3, osd=0)
    for i, c in enumerate(cases):
        c["id"] = i
    return cases


def main():
    cases = build_cases()
    # heaviest first for better packing
    weight = lambda c: c["shots"] * c["max_iter"] * (20 if c["algo"] == "BP" else 1) * \
        (50 if c["sched"] == "S" else 1) * {"LP118_2": 8, "LP118_0": 4}.get(c["code"], 1)
    order = sorted(cases, key=weight, reverse=True)
    results = {}
    with Pool(int(os.environ.get("GOLDEN_PROCS", "8"))) as pool:
        for case, arrs in pool.imap_unordered(run_case, order):
            results[case["id"]] = (case, arrs)
            print(f"[{len(results)}/{len(cases)}] {case['algo']} {case['code']} {case['half']} "
                  f"{case['sched']} {case['kind']} p={case['p_phys']} it={case['max_iter']} "
                  f"osd={case['osd']} iters={arrs['iters'].tolist() if arrs else case.get('raises')}", flush=True)
    groups = {}
    for cid in sorted(results):
        case, arrs = results[cid]
        key = f"{case['algo'].lower()}_{case['code']}" + ("_osd" if case["osd"] >= 0 else "")
        groups.setdefault(key, []).append((case, arrs))
    for key, items in groups.items():
        out = {}
        meta = []
        for i, (case, arrs) in enumerate(items):
            meta.append(case)
            for name, a in arrs.items():  # empty for cases where the reference raises
                out[f"c{i}_{name}"] = a
        out["cases_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
        np.savez_compressed(os.path.join(HERE, f"{key}.npz"), **out)
        print("wrote", key, len(items), "cases")


if __name__ == "__main__":
    main()
