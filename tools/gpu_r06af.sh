# round-6 session: OSD engine issue priority re-checked after the engine-read step (3 / 2 / 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06af osdab:main,op2,op1 || exit 1
echo done
