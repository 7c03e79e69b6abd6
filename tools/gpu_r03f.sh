# round-3 GPU pass f: full GPU suite, then A/B of this round's switches
# (lift-16 flood layout, compressed layered records, OSD engine tickets)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03f_pytest.log 2>&1
rc=$?
tail -15 gpurun_out/r03f_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py QLDPC_FLOOD_PLAIN LP118_0 MS F None 50 524288 3 > gpurun_out/r03f_ab_flood.json 2>&1 || exit 1
tail -3 gpurun_out/r03f_ab_flood.json
timeout -k 10 300 python -u tools/ab_env.py QLDPC_MS_C2V_FULL LP118_2 MS L 0.05 50 262144 3 > gpurun_out/r03f_ab_cc.json 2>&1 || exit 1
tail -3 gpurun_out/r03f_ab_cc.json
timeout -k 10 200 python -u tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 5 > gpurun_out/r03f_osd.json 2>&1 || exit 1
tail -2 gpurun_out/r03f_osd.json
QLDPC_OSD_NO_TICKETS=1 timeout -k 10 200 python -u tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 5 > gpurun_out/r03f_osd_noticket.json 2>&1 || exit 1
tail -2 gpurun_out/r03f_osd_noticket.json
timeout -k 10 300 python -u tools/bench_sim.py 262144 LP118_2:MS > gpurun_out/r03f_sim.json 2>&1 || exit 1
tail -3 gpurun_out/r03f_sim.json
timeout -k 10 400 python -u tools/bench_configs.py > gpurun_out/r03f_configs.jsonl 2>&1 || { tail -5 gpurun_out/r03f_configs.jsonl; exit 1; }
cat gpurun_out/r03f_configs.jsonl
