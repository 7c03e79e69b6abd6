"""Interleaved A/B timing of library builds on one GPU in one process each round.

usage: python tools/ab_bench.py LIB_A LIB_B [...] [--rounds R] [--batch B]
Each round runs every library's headline decode (LP118_0 MS-F 50 it, random
syndromes) in a subprocess, in rotating order; prints per-library median and
min kernel ms per 2^20-equivalent launch.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def main():
    args = sys.argv[1:]
    rounds, batch = 3, 1 << 19
    if "--rounds" in args:
        i = args.index("--rounds"); rounds = int(args[i + 1]); del args[i:i + 2]
    if "--batch" in args:
        i = args.index("--batch"); batch = int(args[i + 1]); del args[i:i + 2]
    libs = args
    res = {l: [] for l in libs}
    for r in range(rounds):
        order = libs[r % len(libs):] + libs[:r % len(libs)]
        for lib in order:
            env = dict(os.environ, QLDPC_LIB=os.path.abspath(lib))
            out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--batch", str(batch),
                                  "--steps", "2", "--warmup", "1", "--cpu-seconds", "0"],
                                 env=env, capture_output=True, text=True, timeout=300)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")]
            if not line:
                print(out.stderr[-2000:])
                raise SystemExit(1)
            d = json.loads(line[-1])
            res[lib].append(d["roofline"]["kernel_ms_per_launch"] * (1 << 20) / batch)
    for lib, v in res.items():
        v = sorted(v)
        print(json.dumps({"lib": os.path.basename(lib), "median_ms": v[len(v) // 2], "min_ms": v[0], "all": v}))


if __name__ == "__main__":
    main()
