# round-6 session: the flooding min-sum kernel in its own max-ILP translation unit —
# A/B against HEAD on every decoder, then the headline parity files
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06q ab:main,h6:head,msl2p10,bpl2p10 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bits.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r06q_parity.log 2>&1; tail -2 gpurun_out/r06q_parity.log
echo done
