"""Interleaved A/B of library builds on tools/prof_sim.py phase times (fresh process per run).
usage: python tools/ab_prof_sim.py ROUNDS "prof_sim args" NAME=LIB [NAME=LIB ...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
rounds, args = int(sys.argv[1]), sys.argv[2].split()
variants = [v.split("=", 1) for v in sys.argv[3:]]
res = {n: {} for n, _ in variants}
for r in range(rounds):
    for name, lib in (variants if r % 2 == 0 else variants[::-1]):
        env = dict(os.environ, QLDPC_LIB=lib)
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof_sim.py")] + args, env=env,
                             capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(out.stderr[-2000:])
            raise SystemExit(1)
        for k, v in json.loads(line[-1])["sec_per_batch"].items():
            res[name].setdefault(k, []).append(round(v * 1e3, 3))
print(json.dumps({"args": args, "ms": {n: {k: sorted(v) for k, v in d.items()} for n, d in res.items()}}))
