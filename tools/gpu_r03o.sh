# round-3 GPU pass o: HBM tile kernel A/B — checks per load step (UC 1 / 2 / 4)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in uc1 uc4 main; do
  lib=qldpcsim_amd/_build/var_hbm_$v.so; [ $v = main ] && lib=qldpcsim_amd/_build/libqldpc_hip.so
  QLDPC_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 python -u tools/bench_configs.py --hbm-large > gpurun_out/r03o_$v.jsonl 2>&1 || { tail -5 gpurun_out/r03o_$v.jsonl; exit 1; }
  echo "== $v"; grep hbm_kernel gpurun_out/r03o_$v.jsonl | python3 -c "import sys,json; [print(round(json.loads(l)['half_shots_per_s']), round(json.loads(l)['hbm_frac'],3)) for l in sys.stdin]"
done
# OSD engine early-exit slot scan: parity, then interleaved A/B vs HEAD's build
timeout -k 10 400 python -u -m pytest tests/test_gpu_osd.py tests/test_gpu_simulator.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03o_osd_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03o_osd_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in head main; do
  lib=qldpcsim_amd/_build/var_head.so; [ $v = main ] && lib=qldpcsim_amd/_build/libqldpc_hip.so
  QLDPC_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 python -u tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 5 > gpurun_out/r03o_osd_$v$r.json 2>&1 || { tail -5 gpurun_out/r03o_osd_$v$r.json; exit 1; }
  echo "$v $(grep osd_shots_per_s gpurun_out/r03o_osd_$v$r.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["sec"]*1e3,2), "ms", d["status_hist"])')"
done; done
