# round-6 session: A/B of the decoder library built without SLP vectorization (the
# layered variable nodes' packed adds needed a register move per packed pair)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06l ab:main,noslp:msl2p10,msl2p05,bpl2p10,bpf0,head || exit 1
echo done
