# round-6 session: check-node reads in one block (the first-iteration branch hoisted out
# of the edge loop) — A/B against HEAD, then the layered / OSD parity files
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06j ab:main,h3:msl2p10,msl2p05,msl0 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_osd.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r06j_parity.log 2>&1; tail -2 gpurun_out/r06j_parity.log
echo done
