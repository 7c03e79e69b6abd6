# round-6 session: the device-memory OSD kernel (codes past the register / LDS kernels):
# the OSD and simulator GPU test files
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_osd.py -m gpu -v -x --timeout 300 --timeout-method thread -k "hbm or large_code or past_the" > gpurun_out/r06u_hbm_osd.log 2>&1; rc=$?; tail -15 gpurun_out/r06u_hbm_osd.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_osd.py tests/test_gpu_simulator.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r06u_osd_all.log 2>&1; rc=$?; tail -3 gpurun_out/r06u_osd_all.log; exit $rc
