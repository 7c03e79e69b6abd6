# round-3 GPU pass ab: layered MS prologue/epilogue with batched loads — parity, interleaved A/B vs HEAD, configs[3] sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bits.py tests/test_gpu_simulator.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03ab_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r03ab_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_libs.py --rounds 3 --cfg "--code LP118_2 --schedule L --p 0.01 --batch 262144 --io bytes" --cfg "--code LP118_2 --schedule L --p 0.05 --batch 262144 --io bytes" --cfg "--code LP118_2 --schedule L --p 0.1 --batch 65536 --io bytes" --cfg "--schedule L --batch 262144" qldpcsim_amd/_build/libqldpc_hip.so qldpcsim_amd/_build/var_head.so > gpurun_out/r03ab_ab.json 2>&1 || { tail -5 gpurun_out/r03ab_ab.json; exit 1; }
cat gpurun_out/r03ab_ab.json
timeout -k 10 600 python -u tools/bench_sim.py 1048576 LP118_2:MS > gpurun_out/r03ab_sim.jsonl 2>&1 || { tail -5 gpurun_out/r03ab_sim.jsonl; exit 1; }
grep shots_per_s gpurun_out/r03ab_sim.jsonl | cut -c1-150
