# round-3 GPU pass v: OSD engine branch-free masked XOR — parity, A/B vs exec-masked build, configs[3] end to end
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_osd.py tests/test_gpu_simulator.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03z_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03z_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in head main; do
  lib=qldpcsim_amd/_build/var_head.so; [ $v = main ] && lib=qldpcsim_amd/_build/libqldpc_hip.so
  QLDPC_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 python -u tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 5 > gpurun_out/r03z_osd_$v$r.json 2>&1 || { tail -5 gpurun_out/r03z_osd_$v$r.json; exit 1; }
  echo "$v $(grep osd_shots_per_s gpurun_out/r03z_osd_$v$r.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["sec"]*1e3,2), "ms", d["status_hist"])')"
done; done
timeout -k 10 300 python -u tools/bench_sim_one.py LP118_2 MS L 0 50 0.1 1048576 > gpurun_out/r03z_sim.json 2>&1 || { tail -5 gpurun_out/r03z_sim.json; exit 1; }
grep shots_per_s gpurun_out/r03z_sim.json | cut -c1-200
