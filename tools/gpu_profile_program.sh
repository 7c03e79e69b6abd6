# Per-kernel counters of an arbitrary python program (GPU box): one
# kernel-trace --stats pass and one --pmc pass per counter set, each its own run.
# usage: bash tools/gpu_profile_program.sh TAG script.py [args...]
#        then python tools/kernel_counters.py TAG  ->  profiles/TAG_kernels.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
PASSES=("FETCH_SIZE"
        "WRITE_SIZE"
        "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE")
D=gpurun_out/kprof_$TAG
mkdir -p $D
echo "$*" > $D/cmd.txt
echo "[$TAG] trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o t -- python3 "$@" > $D/trace.log 2>&1 || { echo "trace failed rc=$?"; tail -5 $D/trace.log; exit 1; }
i=0
for set in "${PASSES[@]}"; do
  i=$((i+1))
  echo "[$TAG] pass $i: $set"
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $D/p$i -o c -- python3 "$@" > $D/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $D/p$i.log; exit 1; }
done
python3 tools/kernel_counters.py $TAG > $D/summary.json 2> $D/summary.err || { cat $D/summary.err; exit 1; }
