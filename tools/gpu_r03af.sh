# round-3 GPU pass af: layered MS — layer-ordered syndrome bits (main vs var_nosynl), layer
# descriptors one layer ahead (var_nosynl vs var_nopf), VN width per layer (var_nopf vs var_h2);
# parity, interleaved A/B, configs[3] sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bits.py tests/test_gpu_simulator.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03af_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r03af_parity.log; [ $rc -eq 0 ] || exit $rc
B=qldpcsim_amd/_build
timeout -k 10 900 python -u tools/ab_libs.py --rounds 3 --cfg "--code LP118_2 --schedule L --p 0.01 --batch 262144 --io bytes" --cfg "--code LP118_2 --schedule L --p 0.05 --batch 262144 --io bytes" --cfg "--code LP118_2 --schedule L --p 0.1 --batch 65536 --io bytes" --cfg "--schedule L --batch 262144" --cfg "--code LP04_0 --schedule L --batch 262144" $B/libqldpc_hip.so $B/var_nosynl.so $B/var_nopf.so $B/var_h2.so > gpurun_out/r03af_ab.json 2>&1 || { tail -5 gpurun_out/r03af_ab.json; exit 1; }
cat gpurun_out/r03af_ab.json
timeout -k 10 600 python -u tools/bench_sim.py 1048576 LP118_2:MS > gpurun_out/r03af_sim.jsonl 2>&1 || { tail -5 gpurun_out/r03af_sim.jsonl; exit 1; }
grep shots_per_s gpurun_out/r03af_sim.jsonl | cut -c1-150
