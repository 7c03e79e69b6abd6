# round-3 GPU pass s: counter profile of the HBM-resident kernel (measured HBM bytes), bench lines with it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_profile_roofline.sh r03s \
  hbm0 "--path hbm --hbm-leg 0 --batch 262144" \
  hbmbp0 "--path hbm --hbm-leg 0 --algo BP --iters 20 --batch 65536" || exit 1
cp gpurun_out/roof_r03s/summary.json profiles/r03s_roofline.json
timeout -k 10 300 python bench.py --path hbm --hbm-leg 0 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/r03s_bench_hbm.log 2>&1 || { tail -5 gpurun_out/r03s_bench_hbm.log; exit 1; }
tail -1 gpurun_out/r03s_bench_hbm.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['bound'], r['frac'], {k:round(v['frac'],3) for k,v in r.get('units',{}).items()})"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r03s_bench.log 2>&1 || { tail -5 gpurun_out/r03s_bench.log; exit 1; }
tail -1 gpurun_out/r03s_bench.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['bound'], r['frac'], json.dumps(d['hbm_streaming'])[:400])"
