# round-6 closing run at HEAD (after the OSD changes): OSD counter profile at its new hash,
# bench (headline + configs[3] / [4] legs), smoke, the full GPU suite, the configs[3] / [4] sweeps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06v roof-osd bench smoke tests sim3 sim4 || exit 1
echo done
