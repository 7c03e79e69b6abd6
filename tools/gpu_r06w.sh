# round-6 session: the wave XOR reduction through row_bcast DPP (one readlane) — A/B
# against the four-readlane form, then the decoder parity files
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06w ab:main,wxold:msl2p10,bpl2p10 parity || exit 1
echo done
