# round-6 session: the two-degree adjacency format (byte offsets, degree by split) in the
# layered MS variable nodes — A/B against HEAD, then the decoder parity files
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06ab ab:main,h9:msl2p10,msl2p05 parity || exit 1
echo done
