set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python tools/ab_bench.py qldpcsim_amd/_build/ab/*.so --rounds 3 > gpurun_out/ab.jsonl 2> gpurun_out/ab.err
