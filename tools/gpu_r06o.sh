# round-6 session: stall attribution of the layered MS kernel after the check-node read fixes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06o stall:main,abl1,abl2:msl2p10 || exit 1
echo done
