# round-6 session: A/B of two lanes per check on <= 32-row layers in the one-lane instance
# (generic split CN; uniform pair CN), the layered parity files on the uniform build, BP stalls
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06f ab:main,mslg2s,mslg2su:msl2p10,msl2p05 || exit 1
QLDPC_LIB=qldpcsim_amd/_build/var_mslg2su.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_osd.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r06f_parity_g2su.log 2>&1; tail -2 gpurun_out/r06f_parity_g2su.log
bash tools/gpu_run.sh r06f stall:main:bpl2p10
echo done
