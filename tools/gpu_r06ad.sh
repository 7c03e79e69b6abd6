# round-6 session: variables per lane per pass on > 128-variable layers (QLDPC_VN_H 2 / 4 / 8)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06ad ab:main,vnh8,vnh2:msl2p10,msl2p05 || exit 1
echo done
