# round-3 GPU pass d: HBM kernel tests + throughput, counter profile (with the
# per-class VALU counters) of the decode kernels, headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hbm.py -v --timeout 120 --timeout-method thread > gpurun_out/r03d_hbm.log 2>&1
rc=$?
tail -12 gpurun_out/r03d_hbm.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/bench_configs.py --hbm > gpurun_out/r03d_hbm_bench.jsonl 2>&1
cat gpurun_out/r03d_hbm_bench.jsonl
bash tools/gpu_profile_roofline.sh r03d \
  flood "" \
  msl2 "--code LP118_2 --schedule L --p 0.05 --batch 262144" \
  bpf0 "--algo BP --iters 100 --batch 65536" \
  bpl2 "--code LP118_2 --algo BP --schedule L --iters 100 --p 0.05 --batch 131072" || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r03d_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r03d_bench.log; exit 1; }
tail -1 gpurun_out/r03d_bench.log
