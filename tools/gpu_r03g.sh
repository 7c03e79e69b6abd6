# round-3 GPU pass g: configs[3] end-to-end phase timing and throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/prof_sim.py LP118_2 MS L 0 50 0.1 131072 > gpurun_out/r03g_profsim.json 2>&1 || { tail -5 gpurun_out/r03g_profsim.json; exit 1; }
tail -3 gpurun_out/r03g_profsim.json
timeout -k 10 300 python -u tools/bench_sim.py 262144 LP118_2:MS > gpurun_out/r03g_sim.json 2>&1 || { tail -5 gpurun_out/r03g_sim.json; exit 1; }
cat gpurun_out/r03g_sim.json
timeout -k 10 400 python -u tools/bench_configs.py --hbm-large > gpurun_out/r03g_hbm_large.jsonl 2>&1 || { tail -5 gpurun_out/r03g_hbm_large.jsonl; exit 1; }
cat gpurun_out/r03g_hbm_large.jsonl
