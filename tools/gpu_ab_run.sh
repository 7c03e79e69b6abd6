# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=ab47
timeout -k 10 500 python -u -m pytest tests/test_gpu_osd.py tests/test_gpu_simulator.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
B=$PWD/qldpcsim_amd/_build
# block-OSD engine: SGPR free masks + uniform pivot-slot switch (new) vs HEAD
for r in 1 2 3; do
  for lib in var_base.so libqldpc_hip.so; do
    QLDPC_LIB=$B/$lib timeout -k 10 120 python -u tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 3 > gpurun_out/${T}_osd_${lib}_$r.log 2>&1 || { tail -5 gpurun_out/${T}_osd_${lib}_$r.log; exit 1; }
    echo "$lib $(grep '^{' gpurun_out/${T}_osd_${lib}_$r.log | tail -1)"
  done
done
