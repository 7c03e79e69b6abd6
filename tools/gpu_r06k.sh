# round-6 session: the one-lane check node's 16 reads under one wait (layered MS), and
# np.prod's permutes issued before the fold (BP team kernels) — A/B against HEAD, parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06k ab:main,h4,bpshfl:msl2p10,msl2p05,bpl2p10,bpf0 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_osd.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r06k_parity.log 2>&1; tail -2 gpurun_out/r06k_parity.log
QLDPC_LIB=qldpcsim_amd/_build/var_bpshfl.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -k "bp or BP" --timeout 200 --timeout-method thread > gpurun_out/r06k_parity_bp.log 2>&1; tail -2 gpurun_out/r06k_parity_bp.log
echo done
