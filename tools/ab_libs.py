"""Interleaved A/B timing of library builds on any bench.py workload.

usage: python tools/ab_libs.py --rounds R --cfg "BENCH ARGS" [--cfg ...] LIB_A LIB_B [...]
Each round runs every (config, library) pair as a fresh bench.py process
(QLDPC_LIB selects the build; LIB@name=v,name=v also sets library options
through QLDPC_OPTIONS), in rotating library order; prints one JSON line
per config with every library's sorted kernel ms per launch (HIP events).
"""
import json
import os
import shlex
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def main():
    args = sys.argv[1:]
    rounds, cfgs = 3, []
    while "--rounds" in args:
        i = args.index("--rounds"); rounds = int(args[i + 1]); del args[i:i + 2]
    while "--cfg" in args:
        i = args.index("--cfg"); cfgs.append(args[i + 1]); del args[i:i + 2]
    cfgs = cfgs or [""]
    libs = args
    for cfg in cfgs:
        res = {l: [] for l in libs}
        kern = {}
        for r in range(rounds):
            order = libs[r % len(libs):] + libs[:r % len(libs)]
            for lib in order:
                path, _, opts = lib.partition("@")
                env = dict(os.environ, QLDPC_LIB=os.path.abspath(path), QLDPC_OPTIONS=opts)
                out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                                      "--cpu-seconds", "0", "--sim-legs", "", "--hbm-leg", "0",
                                      *shlex.split(cfg)],
                                     env=env, capture_output=True, text=True, timeout=300)
                line = [l for l in out.stdout.splitlines() if l.startswith("{")]
                if not line:
                    print(out.stderr[-3000:], flush=True)
                    raise SystemExit(1)
                d = json.loads(line[-1])
                res[lib].append(round(d["roofline"]["kernel_ms_per_launch"], 3))
                kern[os.path.basename(lib)] = d["roofline"].get("kernel")
        print(json.dumps({"cfg": cfg, "kernel_ms": {os.path.basename(k): sorted(v) for k, v in res.items()},
                          "kernel": kern,
                          "avg_it": d["config"]["avg_iterations"]}), flush=True)


if __name__ == "__main__":
    main()
