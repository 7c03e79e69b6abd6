"""Interleaved A/B of a switch on one config (same box, one process per run).
usage: python tools/ab_env.py SWITCH[=VALUE] code algo sched p max_iter batch [rounds]
SWITCH is an environment variable, or a lower-case library option (include/
qldpc_decoder.h, qldpc_set_option), passed as QLDPC_OPTIONS=name=value.
("on" sets it to VALUE, default 1; SWITCH=ON/OFF sets OFF for "off" instead of unsetting)"""
import json
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
env_var, code, algo, sched, p, it, B = sys.argv[1:8]
env_var, _, env_val = env_var.partition("=")
env_val, _, env_off = env_val.partition("/")      # VAR=ON/OFF: "off" sets OFF instead of unsetting
rounds = int(sys.argv[8]) if len(sys.argv) > 8 else 3
snippet = (f"import sys; sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {ROOT + '/tools'!r});"
           f"import bench_configs as b, json; print(json.dumps(b.run({code!r}, {algo!r}, {sched!r}, "
           f"{None if p == 'None' else float(p)}, {int(it)}, {int(B)})))")
res = {"off": [], "on": []}
for r in range(rounds):
    for k in (("off", "on") if r % 2 == 0 else ("on", "off")):
        env = dict(os.environ)
        val = (env_val or "1") if k == "on" else env_off
        if env_var.islower():                                  # a library option
            if val:
                env["QLDPC_OPTIONS"] = f"{env_var}={val}"
        elif val:
            env[env_var] = val
        else:
            env.pop(env_var, None)
        out = subprocess.run([sys.executable, "-c", snippet], env=env, capture_output=True, text=True)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(out.stderr[-2000:]); raise SystemExit(1)
        res[k].append(json.loads(line[-1])["kernel_ms_per_launch"])
print(json.dumps({env_var: {k: sorted(v) for k, v in res.items()}}))
