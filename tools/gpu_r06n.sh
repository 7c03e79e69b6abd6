# round-6 session: the device OSD kernels built without SLP vectorization (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06n osdab:main,noslp || exit 1
echo done
