"""Interleaved A/B/C... of environment variants on one config (fresh process per run).
usage: python tools/ab_variants.py code algo sched p max_iter batch rounds VAR [VAR ...]
  VAR = "name" (no env) or "name:ENV1=1,ENV2=3"; prints one JSON line of sorted
  kernel ms per launch for each variant."""
import json
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
code, algo, sched, p, it, B, rounds = sys.argv[1:8]
variants = []
for v in sys.argv[8:]:
    name, _, envs = v.partition(":")
    env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
    variants.append((name, env))
snippet = (f"import sys; sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {ROOT + '/tools'!r});"
           f"import bench_configs as b, json; print(json.dumps(b.run({code!r}, {algo!r}, {sched!r}, "
           f"{None if p == 'None' else float(p)}, {int(it)}, {int(B)})))")
res = {name: [] for name, _ in variants}
for r in range(int(rounds)):
    order = variants if r % 2 == 0 else variants[::-1]
    for name, extra in order:
        env = dict(os.environ)
        env.update(extra)
        out = subprocess.run([sys.executable, "-c", snippet], env=env, capture_output=True, text=True,
                             timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(out.stderr[-3000:])
            raise SystemExit(1)
        res[name].append(round(json.loads(line[-1])["kernel_ms_per_launch"], 3))
print(json.dumps({"config": [code, algo, sched, p, it, B], "ms": {k: sorted(v) for k, v in res.items()}}),
      flush=True)
