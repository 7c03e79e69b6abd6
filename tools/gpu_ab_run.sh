# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab8_pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/ab8_pytest.log; exit 1; }
tail -2 gpurun_out/ab8_pytest.log
for io in bytes bits; do timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --io $io > gpurun_out/ab8_bench_$io.log 2>&1 || exit 1; python -c "import json;d=json.loads(open('gpurun_out/ab8_bench_$io.log').read().strip().splitlines()[-1]);print('$io',d['value'],d['roofline']['kernel_ms_per_launch'])"; done
timeout -k 10 -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ab8_w -o c -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/ab8_w.log 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ab8_f -o c -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/ab8_f.log 2>&1 || exit 1
