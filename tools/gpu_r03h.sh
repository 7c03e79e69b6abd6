# round-3 GPU pass h: compressed-record layered MS without spills (A/B), parity
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "layered_kernels" --timeout 120 --timeout-method thread > gpurun_out/r03h_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03h_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py QLDPC_MS_CC LP118_2 MS L 0.05 50 262144 3 > gpurun_out/r03h_ab_cc.json 2>&1 || exit 1
tail -1 gpurun_out/r03h_ab_cc.json
timeout -k 10 300 python -u tools/ab_env.py QLDPC_MS_CC LP118_2 MS L 0.1 50 65536 3 > gpurun_out/r03h_ab_cc_p1.json 2>&1 || exit 1
tail -1 gpurun_out/r03h_ab_cc_p1.json
