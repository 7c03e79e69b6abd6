# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=ab24
timeout -k 10 300 python -u tools/prof_osd_path.py LP118_2 MS L 50 0.05 > gpurun_out/${T}.log 2>&1 || { tail -20 gpurun_out/${T}.log; exit 1; }
grep -v "^$" gpurun_out/${T}.log | head -45
timeout -k 10 600 python -u tools/bench_sim.py 1048576 LP118_2:MS > gpurun_out/sim_$T.jsonl 2> gpurun_out/sim_$T.err || { tail -5 gpurun_out/sim_$T.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/sim_$T.jsonl'):
    d=json.loads(l); print(d['p'], round(d['shots_per_s']/1e6,3))"
