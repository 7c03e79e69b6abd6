# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=ab17
QLDPC_OSD_PROF=1 QLDPC_LIB=$PWD/qldpcsim_amd/_build/var_prof.so timeout -k 10 300 python tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 2 > gpurun_out/${T}.log 2>&1 || { tail -20 gpurun_out/${T}.log; exit 1; }
grep osd_prof gpurun_out/${T}.log | tail -3; tail -1 gpurun_out/${T}.log
