set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_bp.py > gpurun_out/diag.log 2>&1
