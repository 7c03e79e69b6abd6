# SQ counter passes on a reduced headline batch (2^18 shots), one --pmc pass each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ctr
rocprofv3 -L > gpurun_out/ctr/counters_list.txt 2>&1 || true
B="python3 bench.py --batch 262144 --steps 1 --warmup 0 --cpu-seconds 0"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64" \
           "SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d gpurun_out/ctr/p$i -o c -- $B > gpurun_out/ctr/p$i.log 2>&1 || echo "pass $i failed rc=$?" >> gpurun_out/ctr/fail.txt
done
exit 0
