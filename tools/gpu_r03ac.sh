# round-3 GPU pass ac: configs[3] p = 0.1 phase timing and per-kernel counters at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/prof_sim.py LP118_2 MS L 0 50 0.1 131072 > gpurun_out/r03ac_phases.json 2>&1 || { tail -5 gpurun_out/r03ac_phases.json; exit 1; }
cat gpurun_out/r03ac_phases.json
bash tools/gpu_profile_program.sh r03ac_cfg3 tools/prof_sim.py LP118_2 MS L 0 50 0.1 131072 && python3 -c "
import json;d=json.load(open('gpurun_out/kprof_r03ac_cfg3/summary.json'))
for k in d['kernels']: print(k['kernel'], round(k['total_ms'],1), k['calls'], k.get('busy'))"
