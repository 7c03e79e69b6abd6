# round-3 GPU pass i: per-phase cycles of osd_block_kernel (diagnostic build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
QLDPC_LIB=$GRAFT_REPO_ROOT/diag/libqldpc_osdprof.so QLDPC_OSD_PROF=1 timeout -k 10 200 python -u tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 1 > gpurun_out/r03i_osdprof.log 2>&1 || { tail -5 gpurun_out/r03i_osdprof.log; exit 1; }
tail -4 gpurun_out/r03i_osdprof.log
