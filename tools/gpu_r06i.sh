# round-6 session: A/B of prefetching the first variable-node trip's adjacency words
# (and their filter words) at the layer head, before the check nodes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06i ab:main,h2,vnpf,vnpfav:msl2p10,msl2p05 || exit 1
echo done
