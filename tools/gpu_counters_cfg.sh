# SQ counter passes for one decoder config (tools/decode_once.py), one --pmc pass each.
# usage: bash tools/gpu_counters_cfg.sh TAG CODE ALGO SCHED P ITERS BATCH
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
D=gpurun_out/ctr_$TAG
mkdir -p $D
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FP64 SQ_INSTS_BRANCH SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $D/p$i -o c -- python3 tools/decode_once.py "$@" > $D/p$i.log 2>&1 || { echo "pass $i failed rc=$?" >> $D/fail.txt; exit 1; }
done
