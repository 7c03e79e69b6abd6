# compact flooding kernel: parity first, then interleaved A/B against the v2 kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "F and MS" > gpurun_out/pytest_fc.log 2>&1 || exit $?
timeout -k 10 900 python tools/ab_variants.py LP118_0 MS F None 50 1048576 3 compact v2:QLDPC_FLOOD_V2=1 noreg:QLDPC_FC_NOREG=1 > gpurun_out/ab_fc.jsonl 2> gpurun_out/ab_fc.err || exit $?
timeout -k 10 600 python tools/ab_variants.py LP04_0 MS F 0.05 50 1048576 2 compact v2:QLDPC_FLOOD_V2=1 noreg:QLDPC_FC_NOREG=1 >> gpurun_out/ab_fc.jsonl 2>> gpurun_out/ab_fc.err || exit $?
timeout -k 10 600 python tools/ab_variants.py LP118_2 MS F None 50 262144 2 compact v2:QLDPC_FLOOD_V2=1 noreg:QLDPC_FC_NOREG=1 >> gpurun_out/ab_fc.jsonl 2>> gpurun_out/ab_fc.err || exit $?
