# round-3 GPU pass ah: full GPU suite at HEAD, smoke, bench, configs[3] / configs[4] sweeps,
# osd_block_kernel per-phase cycles (QLDPC_OSD_TIMING build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r03ah_pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r03ah_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ah_smoke.log 2>&1 || { tail -8 gpurun_out/r03ah_smoke.log; exit 1; }
tail -2 gpurun_out/r03ah_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r03ah_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r03ah_bench.log; exit 1; }
tail -1 gpurun_out/r03ah_bench.log | cut -c1-300
timeout -k 10 600 python -u tools/bench_sim.py 1048576 LP118_2:MS > gpurun_out/r03ah_sim_cfg3.jsonl 2>&1 || { tail -5 gpurun_out/r03ah_sim_cfg3.jsonl; exit 1; }
grep shots_per_s gpurun_out/r03ah_sim_cfg3.jsonl | cut -c1-150
QLDPC_LIB=qldpcsim_amd/_build/var_otime.so QLDPC_OSD_PROF=1 timeout -k 10 300 python -u tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 3 > gpurun_out/r03ah_osd_prof.log 2>&1 || { tail -5 gpurun_out/r03ah_osd_prof.log; exit 1; }
grep -v "^$" gpurun_out/r03ah_osd_prof.log | tail -8
