# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=ab31
timeout -k 10 600 python -u -m pytest tests/test_gpu_osd.py tests/test_gpu_simulator.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
B=$PWD/qldpcsim_amd/_build
timeout -k 10 600 python -u tools/ab_libs.py --rounds 3 --cfg "--algo BP --iters 100 --batch 65536" --cfg "--code LP118_2 --algo BP --schedule L --iters 100 --p 0.05 --batch 131072" --cfg "--algo BP --iters 100 --p 0.05 --batch 262144" $B/var_base.so $B/libqldpc_hip.so > gpurun_out/${T}_ab.log 2>&1 || { tail -20 gpurun_out/${T}_ab.log; exit 1; }
cat gpurun_out/${T}_ab.log | grep "{"
timeout -k 10 600 python -u tools/bench_sim.py 1048576 LP118_2:MS > gpurun_out/sim_$T.jsonl 2> gpurun_out/sim_$T.err || { tail -5 gpurun_out/sim_$T.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/sim_$T.jsonl'):
    d=json.loads(l); print(d['p'], round(d['shots_per_s']/1e6,3))"
