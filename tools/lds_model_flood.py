"""LDS bank model of ms_flood_kernel's per-iteration LDS traffic, from the
MI355X LDS table (MI355X_MICROARCH.md §LDS: lane groups per instruction,
bank = (a/4) mod 32 or 64, one LDS-array cycle per distinct dword address on
the busiest bank of a group). Recomputes the tables capi.cpp builds (degree
relabeling, CSC positions, row words) and counts array cycles per
wave-iteration: check node (8 post reads b64 + 8 c2v reads b32 + 8 c2v writes
b32 per check slot) and variable node (K c2v reads b32 per run chunk + one
post write b64). Used to pick conflict-free check / edge / variable orders.

Usage: python tools/lds_model_flood.py [code]
"""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))


def relabel(H):
    deg = H.sum(0)
    vperm = np.argsort(deg, kind="stable")
    vinv = np.empty_like(vperm)
    vinv[vperm] = np.arange(len(vperm))
    return vperm, vinv


def tables(H, vperm=None, check_order=None, edge_key=None):
    """post byte offsets pa[c][k], c2v byte offsets ca[c][k] (k < deg), and
    VN runs, for a given variable relabeling (vperm: label -> original)."""
    m, n = H.shape
    if vperm is None:
        vperm, vinv = relabel(H)
    else:
        vinv = np.empty_like(vperm)
        vinv[vperm] = np.arange(n)
    deg = H.sum(0)[vperm]
    csc_ptr = np.concatenate([[0], np.cumsum(deg)])
    fill = csc_ptr[:-1].copy()
    rows = [np.flatnonzero(H[r]) for r in range(m)]
    pos = {}
    for r in range(m):                                  # CSR order: ascending check, then variable
        for j in rows[r]:
            v = vinv[j]
            pos[(r, j)] = fill[v]
            fill[v] += 1
    pa, ca = [], []
    for r in range(m):
        js = list(rows[r])
        if edge_key is not None:
            js.sort(key=lambda j: edge_key(r, j))
        pa.append([8 * vinv[j] for j in js])
        ca.append([4 * pos[(r, j)] for j in js])
    runs = []
    j = 0
    while j < n:
        e = j
        while e < n and deg[e] == deg[j]:
            e += 1
        runs.append((j, e - j, int(deg[j]), int(csc_ptr[j])))
        j = e
    return pa, ca, runs, int(csc_ptr[-1])


def group_cycles(addrs, nbank, lanes_per_group, dwords):
    """addrs: byte address per lane (None = inactive). Cycles = sum over lane
    groups of max over banks of distinct dword addresses."""
    tot = 0
    for g0 in range(0, 64, lanes_per_group):
        banks = {}
        for a in addrs[g0:g0 + lanes_per_group]:
            if a is None:
                continue
            for d in range(dwords):
                w = a // 4 + d
                banks.setdefault(w % nbank, set()).add(w)
        tot += max([len(s) for s in banks.values()] + [1])
    return tot


def flood_cycles(H, pa, ca, runs, E, slots=None):
    """LDS-array cycles per wave-iteration. slots[i][lane] = check index or -1 (pad)."""
    m = H.shape[0]
    KC = (m + 63) // 64
    if slots is None:
        slots = [[(l + 64 * i) if l + 64 * i < m else -1 for l in range(64)] for i in range(KC)]
    cn = {"post_b64": 0, "c2v_rd_b32": 0, "c2v_wr_b32": 0}
    for i in range(len(slots)):
        for k in range(8):
            pp = [8 * 0 if c < 0 else (pa[c][k] if k < len(pa[c]) else None) for c in slots[i]]
            cc = [4 * (E + k) if c < 0 else (ca[c][k] if k < len(ca[c]) else None) for c in slots[i]]
            if all(x is None for x in pp):
                continue
            cn["post_b64"] += group_cycles(pp, 64, 32, 2)
            cn["c2v_rd_b32"] += group_cycles(cc, 32, 32, 1)
            cn["c2v_wr_b32"] += group_cycles(cc, 32, 32, 1)
    vn = {"c2v_rd_b32": 0, "post_wr_b64": 0}
    for (st, cnt, K, p0) in runs:
        for o0 in range(0, cnt, 64):
            lanes = [o0 + l if o0 + l < cnt else None for l in range(64)]
            for t in range(K):
                vn["c2v_rd_b32"] += group_cycles([None if o is None else 4 * (p0 + o * K + t) for o in lanes], 32, 32, 1)
            vn["post_wr_b64"] += group_cycles([None if o is None else 8 * (st + o) for o in lanes], 32, 16, 2)
    return cn, vn


def main():
    from qldpcsim_amd import codes
    name = sys.argv[1] if len(sys.argv) > 1 else "LP118_0"
    Hx, Hz = codes.load_code(name)
    for half, H in (("X (Hz)", Hz), ("Z (Hx)", Hx)):
        pa, ca, runs, E = tables(H.astype(np.int64))
        cn, vn = flood_cycles(H, pa, ca, runs, E)
        print(half, "CN", cn, sum(cn.values()), "VN", vn, sum(vn.values()), "total", sum(cn.values()) + sum(vn.values()))


if __name__ == "__main__":
    main()
