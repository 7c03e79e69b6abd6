# round-3 GPU pass aj: configs[4] (LP118_2 BP-L) end-to-end sweep at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/bench_sim.py 1048576 LP118_2:BP > gpurun_out/r03aj_sim_cfg4.jsonl 2>&1 || { tail -5 gpurun_out/r03aj_sim_cfg4.jsonl; exit 1; }
grep shots_per_s gpurun_out/r03aj_sim_cfg4.jsonl | cut -c1-150
