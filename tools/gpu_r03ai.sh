# round-3 GPU pass ai: osd_block_kernel at 3 waves per SIMD (164 VGPRs, no spills) vs 4 (128, spills), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B=qldpcsim_amd/_build
QLDPC_LIB=$B/var_wpe3.so timeout -k 10 200 python -u -m pytest tests/test_gpu_osd.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ai_osd_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03ai_osd_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in libqldpc_hip.so var_wpe3.so; do
    QLDPC_LIB=$B/$lib timeout -k 10 200 python -u tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 3 > gpurun_out/r03ai_$lib.$r.json 2>&1 || { tail -5 gpurun_out/r03ai_$lib.$r.json; exit 1; }
    echo "$lib $(tail -1 gpurun_out/r03ai_$lib.$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["sec"]*1e3,2), "ms", d["status_hist"])')"
  done
done
