# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=ab55
B=$PWD/qldpcsim_amd/_build
timeout -k 10 300 python -u -m pytest tests/test_gpu_osd.py tests/test_gpu_simulator.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
# block-OSD at 5 waves per SIMD vs 4 (default)
for r in 1 2 3; do
  for lib in libqldpc_hip.so var_wpe5.so; do
    QLDPC_LIB=$B/$lib timeout -k 10 120 python -u tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 3 > gpurun_out/${T}_osd_${lib}_$r.log 2>&1 || { tail -5 gpurun_out/${T}_osd_${lib}_$r.log; exit 1; }
    echo "$lib $(grep '^{' gpurun_out/${T}_osd_${lib}_$r.log | tail -1 | cut -c1-200)"
  done
done
