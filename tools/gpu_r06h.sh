# round-6 session: A/B of the two-degree variable-node sums and the v_min pad clamps in
# the layered MS kernel; the layered / OSD parity files on the new default build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06h ab:main,hbase,notwo:msl2p10,msl2p05 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_osd.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r06h_parity.log 2>&1; tail -2 gpurun_out/r06h_parity.log
echo done
