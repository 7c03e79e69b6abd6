# round-6 session: layered MS check nodes read their syndrome bit by layer position
# (synl, built once per half-shot; the lane-group instance only) — A/B against HEAD, parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06y ab:main,h8:msl0,msl2p10 parity || exit 1
echo done
