# round-6 closing run at the final kernels: layered MS counter profile at its final hash,
# per-config bench lines, bench, smoke, the full GPU suite, the configs[3] / [4] sweeps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06ac roof-msl bench-cfg bench smoke tests sim3 sim4 || exit 1
echo done
