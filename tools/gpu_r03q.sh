# round-3 GPU pass q: OSD host orders on a worker thread (simulator pipeline) — tests, configs[3] end to end + trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_osd.py tests/test_gpu_simulator.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03q_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/probe_host_order.py 23000 > gpurun_out/r03q_host_order.json 2>&1; tail -1 gpurun_out/r03q_host_order.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03q_simtrace -o s -- python3 tools/bench_sim_one.py LP118_2 MS L 0 50 0.1 1048576 > gpurun_out/r03q_simtrace.log 2>&1 || { tail -5 gpurun_out/r03q_simtrace.log; exit 1; }
grep shots_per_s gpurun_out/r03q_simtrace.log | cut -c1-200
timeout -k 10 600 python -u tools/bench_sim.py 1048576 LP118_2:MS > gpurun_out/r03q_sim.jsonl 2>&1 || { tail -5 gpurun_out/r03q_sim.jsonl; exit 1; }
grep shots_per_s gpurun_out/r03q_sim.jsonl | cut -c1-160
