# round-6 closing profiles and run at HEAD (after the wave-XOR step): counter profiles of
# the layered MS and BP kernels at their new hashes, the per-config bench lines, bench,
# smoke, the full GPU suite and the configs[3] / [4] sweeps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06x roof-msl roof-bp bench-cfg bench smoke tests sim3 sim4 || exit 1
echo done
