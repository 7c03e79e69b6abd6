# round-6 closing profiles: counter profiles of the headline, layered MS and BP kernels at
# their HEAD machine-code hashes (bench.py's roofline matches them by hash)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06r roof-flood roof-msl roof-bp || exit 1
echo done
