# round-6 session: layered variable-node prefix sums through inline-asm v_add_f32 (no SLP
# pairing into v_pk_add_f32 with register moves) — A/B, then the layered parity files on it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06aa ab:main,vadd:msl2p10,msl2p05 || exit 1
QLDPC_LIB=qldpcsim_amd/_build/var_vadd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_osd.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r06aa_parity_vadd.log 2>&1; rc=$?; tail -2 gpurun_out/r06aa_parity_vadd.log; exit $rc
