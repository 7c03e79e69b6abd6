set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B=qldpcsim_amd/_build
timeout -k 10 300 python -u -m pytest tests/test_gpu_simulator.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_abc.log 2>&1 || exit $?
timeout -k 10 600 python tools/ab_prof_sim.py 3 "LP118_0 MS F -1 50 0.01 262144" head=$B/var_head.so new=$B/var_new.so > gpurun_out/ab_chan.jsonl 2> gpurun_out/ab_chan.err || exit $?
timeout -k 10 600 python tools/ab_prof_sim.py 3 "LP118_2 MS L 0 50 0.05 262144" head=$B/var_head.so new=$B/var_new.so >> gpurun_out/ab_chan.jsonl 2>> gpurun_out/ab_chan.err || exit $?
