# round-6 closing run at HEAD: bench (headline + configs[3] / [4] legs), smoke, the full
# GPU suite, the configs[3] / [4] p-sweeps and the per-config bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06s bench smoke tests sim3 sim4 bench-cfg || exit 1
echo done
