# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=ab53
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 600 python -u tools/bench_sim.py 1048576 LP118_2:BP > gpurun_out/${T}_sim.jsonl 2> gpurun_out/${T}_sim.err || { tail -5 gpurun_out/${T}_sim.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/${T}_sim.jsonl'):
    d=json.loads(l); print(d['code'], d['decType'], d['p'], round(d['shots_per_s']/1e6,3), d['qBLER'])"
