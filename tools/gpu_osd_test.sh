set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_osd.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_configs.py --osd > gpurun_out/osd_rate.jsonl 2>> gpurun_out/osd_rate.err || exit $?
timeout -k 10 300 python tools/prof_sim.py LP118_2 MS L 0 50 0.1 > gpurun_out/prof_sim_osd.jsonl 2>> gpurun_out/osd_rate.err || exit $?
