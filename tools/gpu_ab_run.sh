# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_configs.py --osd 2>&1 | tee gpurun_out/ab7_osd.jsonl || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/ab7_pmc -o c -- python3 tools/bench_configs.py --osd > gpurun_out/ab7_pmc.log 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS --output-format csv -d gpurun_out/ab7_pmc2 -o c -- python3 tools/bench_configs.py --osd > gpurun_out/ab7_pmc2.log 2>&1 || exit 1
