# round-6 final check at HEAD: the full GPU suite, smoke, bench, and a fresh counter
# profile of the HBM-resident kernel (hash unchanged since round 4)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06z tests smoke bench roof-hbm || exit 1
echo done
