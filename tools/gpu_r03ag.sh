# round-3 GPU pass ag: osd_block_kernel per-phase cycles (QLDPC_OSD_TIMING build) on configs[3] p = 0.1 inputs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
QLDPC_LIB=qldpcsim_amd/_build/var_otime.so QLDPC_OSD_PROF=1 timeout -k 10 300 python -u tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 3 > gpurun_out/r03ag_osd_prof.log 2>&1 || { tail -5 gpurun_out/r03ag_osd_prof.log; exit 1; }
grep -v "^$" gpurun_out/r03ag_osd_prof.log | tail -12
