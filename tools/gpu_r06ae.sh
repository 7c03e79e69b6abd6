# round-6 session: layered MS phase priorities re-checked at the final kernel (none / CN at 1 / VN at 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06ae ab:main,pr0,pr2:msl2p10,msl2p05 || exit 1
echo done
