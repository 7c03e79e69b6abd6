# round-3 GPU pass k: roofline profile keyed by per-kernel code hashes, per-kernel
# counters of the configs[3] pipeline (sampler, layered MS, OSD order/elimination, counters), bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_profile_roofline.sh r03k \
  flood "" \
  msl2 "--code LP118_2 --schedule L --p 0.05 --batch 262144" \
  bpf0 "--algo BP --iters 100 --batch 65536" \
  bpl2 "--code LP118_2 --algo BP --schedule L --iters 100 --p 0.05 --batch 131072" || exit 1
bash tools/gpu_profile_program.sh r03k_cfg3 tools/prof_sim.py LP118_2 MS L 0 50 0.1 131072 || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r03k_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r03k_bench.log; exit 1; }
tail -1 gpurun_out/r03k_bench.log
