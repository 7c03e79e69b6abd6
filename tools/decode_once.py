"""One decode launch per half of a config (for rocprofv3 counter passes).
usage: python tools/decode_once.py CODE ALGO SCHED P ITERS BATCH"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_configs as b  # noqa: E402

code, algo, sched, p, it, B = sys.argv[1:7]
b.run(code, algo, sched, None if p == "None" else float(p), int(it), int(B), reps=1)
