# round-6 session: BP team kernels in their own translation unit without SLP
# vectorization — A/B against HEAD, then the full GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06m ab:main,h5:bpl2p10,bpf0,msl2p10,head tests || exit 1
echo done
