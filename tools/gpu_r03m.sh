# round-3 GPU pass l: tiled HBM kernel — tests, throughput (small and chip-filling batches)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hbm.py -v -x --timeout 200 --timeout-method thread > gpurun_out/r03m_hbm.log 2>&1
rc=$?; tail -12 gpurun_out/r03m_hbm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_configs.py --hbm > gpurun_out/r03m_hbm_bench.jsonl 2>&1 || { tail -5 gpurun_out/r03m_hbm_bench.jsonl; exit 1; }
cat gpurun_out/r03m_hbm_bench.jsonl
timeout -k 10 300 python -u tools/bench_configs.py --hbm-large > gpurun_out/r03m_hbm_large.jsonl 2>&1 || { tail -5 gpurun_out/r03m_hbm_large.jsonl; exit 1; }
cat gpurun_out/r03m_hbm_large.jsonl
