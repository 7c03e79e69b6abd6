# round-6 session: OSD 16-word instance A/B; full suite, layered-MS profile and the
# configs[3] / configs[4] sweeps at the new default kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06g osdab:main,osdnw16 tests roof-msl sim3 sim4 || exit 1
echo done
