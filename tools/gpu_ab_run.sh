# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_osd.py tests/test_gpu_simulator.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab5_pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/ab5_pytest.log; exit 1; }
tail -2 gpurun_out/ab5_pytest.log
cat > /tmp/sim5.py <<'PY'
import json, os, sys, time
sys.path.insert(0, os.getcwd())
from qldpcsim_amd import codes, simulator
Hx, Hz = codes.load_code("LP118_2")
for p in (0.05, 0.1):
    for env in ("0", "1"):
        os.environ["QLDPC_OSD_HOST_ORDER"] = env
        kw = dict(shots=1 << 20, decType="MS", decIterations=50, decSchedule="L", OSDorder=0, verbose=False)
        simulator.simulate_p(Hx, Hz, p, rngSeed=2, **kw)
        t0 = time.perf_counter()
        r = simulator.simulate_p(Hx, Hz, p, rngSeed=1, **kw)
        dt = time.perf_counter() - t0
        print(json.dumps({"p": p, "host_order_only": env, "shots_per_s": (1 << 20) / dt, **r}), flush=True)
PY
timeout -k 10 600 python /tmp/sim5.py 2>&1 | tee gpurun_out/ab5_sim.jsonl || exit 1
