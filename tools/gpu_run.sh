# One parametrised GPU-box session (replaces the per-pass gpu_r0*.sh scripts).
# usage: bash tools/gpu_run.sh TAG STEP [STEP ...]
# steps (each under its own time limit; the session stops at the first failure):
#   tests          full `pytest -m gpu`                       -> gpurun_out/TAG_pytest_gpu.log
#   parity         decoder parity subset (parity, bits, osd)  -> gpurun_out/TAG_parity.log
#   smoke          __graft_entry__.smoke()                    -> gpurun_out/TAG_smoke.log
#   bench          bench.py --steps 20 --warmup 5 (headline)  -> gpurun_out/TAG_bench.log
#   bench-cfg      bench.py on the configs[2]-[4] decoders    -> gpurun_out/TAG_bench_cfg.jsonl
#   roof-decoders  counter profile (tools/gpu_profile_roofline.sh) of the configs[2]-[4] decoders
#   roof-bp / roof-msl  counter profiles of the BP decoders / the layered MS decoder only
#   roof-osd       counter profile of the device OSD kernels (tools/osd_bench.py, configs[3] p = 0.1)
#   roof-flood     counter profile of the headline kernel
#   roof-hbm       counter profile of the HBM-resident kernel on the headline workload
#   sim3 / sim4    tools/bench_sim.py p-sweep of configs[3] / configs[4]
#   phases3/4      tools/prof_sim.py phase times of one configs[3] / configs[4] p = 0.1 batch
#   ties           tools/osd_tie_stats.py: near-tie positions by OSD status (configs[3] p = 0.1)
#   cfg3trace      rocprofv3 kernel trace + stats of tools/prof_sim.py on configs[3] p = 0.1
#   sim3trace      rocprofv3 kernel + copy trace of one configs[3] p = 0.1 simulate_p run (tools/bench_sim_one.py)
#   cfg3prof       per-kernel counters of one configs[3] p = 0.1 batch (tools/gpu_profile_program.sh)
#   osd            tools/osd_bench.py on the configs[3] p = 0.1 OSD shots
#   osdab:LIBS     interleaved A/B of the device OSD (tools/osd_bench.py, configs[3] p = 0.1) over library builds
#   simab:LIBS     configs[3] sweep (tools/bench_sim.py) per library build, two interleaved rounds
#   stall:LIBS:CFG SQ wave-state counters (WAIT_ANY / WAIT_INST_ANY / ACTIVE_*) per build, one cfg preset
#   ab:LIBS:CFGS   interleaved A/B (tools/ab_libs.py) of qldpcsim_amd/_build/var_<name>.so builds;
#                  LIBS = comma-separated names (main = the in-tree build; name+opt=v+opt=v adds
#                  library options), CFGS = cfg preset names
#                  (flood, msl2p05, msl2p10, msl0, bpl2p10, bpl2p05, bpf0, hbm) joined by commas
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
O=gpurun_out
B=qldpcsim_amd/_build

declare -A CFG=(
  [flood]=""
  [msl2p01]="--code LP118_2 --schedule L --p 0.01 --batch 1048576"
  [msl2p05]="--code LP118_2 --schedule L --p 0.05 --batch 262144"
  [msl2p10]="--code LP118_2 --schedule L --p 0.1 --batch 131072"
  [msl0]="--schedule L --batch 262144"
  [bpl2p10]="--code LP118_2 --algo BP --schedule L --iters 100 --p 0.1 --batch 65536"
  [bpl2p01]="--code LP118_2 --algo BP --schedule L --iters 100 --p 0.01 --batch 524288"
  [bpl2p05]="--code LP118_2 --algo BP --schedule L --iters 100 --p 0.05 --batch 131072"
  [bpf0]="--algo BP --iters 100 --batch 65536"
  [hbm]="--path hbm --batch 262144 --hbm-leg 0"
)

fail() { echo "[$TAG] step $1 failed (rc=$2)"; [ -n "$3" ] && tail -8 "$3"; exit 1; }

for step in "$@"; do
  echo "[$TAG] $step"
  case $step in
    tests)
      L=$O/${TAG}_pytest_gpu.log
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $L 2>&1 || fail $step $? $L
      tail -2 $L ;;
    parity)
      L=$O/${TAG}_parity.log
      timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bits.py tests/test_gpu_osd.py -m gpu -x -q \
        --timeout 200 --timeout-method thread > $L 2>&1 || fail $step $? $L
      tail -2 $L ;;
    smoke)
      L=$O/${TAG}_smoke.log
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $L 2>&1 || fail $step $? $L
      tail -2 $L ;;
    bench)
      L=$O/${TAG}_bench.log
      timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $L 2>&1 || fail $step $? $L
      tail -1 $L | cut -c1-300 ;;
    bench-cfg)
      L=$O/${TAG}_bench_cfg.jsonl
      : > $L
      for c in msl2p05 msl2p10 bpl2p10 bpf0; do
        timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --hbm-leg 0 ${CFG[$c]} >> $L 2> $O/${TAG}_bench_cfg.err || fail $step $? $O/${TAG}_bench_cfg.err
      done
      python3 -c "
import json,sys
for l in open('$L'):
    d=json.loads(l); r=d['roofline']
    print(d['config']['code'],d['config']['algo'],d['config']['schedule'],d['config']['p'],round(d['value']/1e6,3),'M', r['kernel'], r['bound'], r['frac'] and round(r['frac'],3))" ;;
    roof-decoders)
      bash tools/gpu_profile_roofline.sh $TAG msl2p05 "${CFG[msl2p05]}" msl2p10 "${CFG[msl2p10]}" \
        bpl2p10 "${CFG[bpl2p10]}" bpf0 "${CFG[bpf0]}" || fail $step $? ;;
    roof-bp)
      bash tools/gpu_profile_roofline.sh ${TAG}b bpl2p10 "${CFG[bpl2p10]}" bpf0 "${CFG[bpf0]}" || fail $step $? ;;
    roof-msl)
      bash tools/gpu_profile_roofline.sh ${TAG}m msl2p05 "${CFG[msl2p05]}" msl2p10 "${CFG[msl2p10]}" || fail $step $? ;;
    roof-osd)
      bash tools/gpu_profile_roofline.sh ${TAG}o osd3p10 "osd:LP118_2 MS L 50 0.1 131072 0 2" || fail $step $? ;;
    roof-flood)
      bash tools/gpu_profile_roofline.sh ${TAG}f flood "" || fail $step $? ;;
    roof-hbm)
      bash tools/gpu_profile_roofline.sh ${TAG}h hbm "${CFG[hbm]}" || fail $step $? ;;
    sim3|sim4)
      L=$O/${TAG}_${step}.jsonl
      [ $step = sim3 ] && W=LP118_2:MS || W=LP118_2:BP
      timeout -k 10 700 python -u tools/bench_sim.py 1048576 $W > $L 2>&1 || fail $step $? $L
      grep shots_per_s $L | cut -c1-160 ;;
    phases3)
      L=$O/${TAG}_phases3.json
      timeout -k 10 300 python -u tools/prof_sim.py LP118_2 MS L 0 50 0.1 131072 > $L 2>&1 || fail $step $? $L ;;
    phases4)
      L=$O/${TAG}_phases4.json
      timeout -k 10 300 python -u tools/prof_sim.py LP118_2 BP L 4 100 0.1 65536 > $L 2>&1 || fail $step $? $L ;;
    phases4b)
      L=$O/${TAG}_phases4b.json
      timeout -k 10 300 python -u tools/prof_sim.py LP118_2 BP L 4 100 0.1 262144 > $L 2>&1 || fail $step $? $L ;;
    ties)
      L=$O/${TAG}_ties.json
      timeout -k 10 200 python -u tools/osd_tie_stats.py LP118_2 MS L 50 0.1 131072 > $L 2>&1 || fail $step $? $L
      tail -1 $L | cut -c1-400 ;;
    cfg3trace)
      D=$O/${TAG}_cfg3trace
      mkdir -p $D
      (export TMPDIR=/tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o t -- \
        python3 tools/prof_sim.py LP118_2 MS L 0 50 0.1 131072 > $D/run.log 2>&1) || fail $step $? $D/run.log
      tail -1 $D/run.log | cut -c1-300 ;;
    sim3trace)
      D=$O/${TAG}_sim3trace
      mkdir -p $D
      (export TMPDIR=/tmp; timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D -o t -- \
        python3 tools/bench_sim_one.py LP118_2 MS L 0 50 0.1 1048576 > $D/run.log 2>&1) || fail $step $? $D/run.log
      tail -1 $D/run.log | cut -c1-200 ;;
    cfg3prof)
      bash tools/gpu_profile_program.sh ${TAG}_cfg3 tools/prof_sim.py LP118_2 MS L 0 50 0.1 131072 || fail $step $? ;;
    osd)
      L=$O/${TAG}_osd.log
      timeout -k 10 300 python -u tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 5 > $L 2>&1 || fail $step $? $L
      tail -4 $L ;;
    osdab:*)
      IFS=: read -r _ libs <<< "$step"
      L=$O/${TAG}_osdab_${libs//,/_}.jsonl
      : > $L
      for r in 1 2 3; do
        for l in ${libs//,/ }; do
          [ $l = main ] && P=$B/libqldpc_hip.so || P=$B/var_$l.so
          QLDPC_LIB=$P timeout -k 10 200 python -u tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 5 >> $L 2>> $O/${TAG}_osdab.err || fail $step $? $O/${TAG}_osdab.err
        done
      done
      python3 -c "
import json,collections
d=collections.defaultdict(list); sh=collections.defaultdict(set)
for l in open('$L'):
    x=json.loads(l); d[x['lib']].append(round(x['sec']*1e3,2)); sh[x['lib']].add((x['ehat_sha'], str(x['status_hist'])))
for k in d: print(k, sorted(d[k]), sh[k])" ;;
    simab:*)
      # configs[3] sweep (tools/bench_sim.py) per library build, two rounds
      IFS=: read -r _ libs <<< "$step"
      L=$O/${TAG}_simab_${libs//,/_}.jsonl
      : > $L
      for r in 1 2; do
        for l in ${libs//,/ }; do
          [ $l = main ] && P=$B/libqldpc_hip.so || P=$B/var_$l.so
          echo "{\"lib\": \"$l\", \"round\": $r}" >> $L
          QLDPC_LIB=$P timeout -k 10 400 python -u tools/bench_sim.py 1048576 LP118_2:MS >> $L 2>> $O/${TAG}_simab.err || fail $step $? $O/${TAG}_simab.err
        done
      done
      grep -o '"lib": "[a-z0-9]*"\|"p": [0-9.]*\|"shots_per_s": [0-9.]*' $L | paste -sd' ' | sed 's/"lib"/\n"lib"/g' ;;
    ab:*)
      IFS=: read -r _ libs cfgs <<< "$step"
      A=()
      for l in ${libs//,/ }; do
        # name+opt=v+opt=v: library options for that entry (QLDPC_OPTIONS)
        n=${l%%+*}; o=; [ "$n" != "$l" ] && o=@${l#*+} && o=${o//+/,}
        [ $n = main ] && A+=($B/libqldpc_hip.so$o) || A+=($B/var_$n.so$o)
      done
      C=()
      for c in ${cfgs//,/ }; do C+=(--cfg "${CFG[$c]}"); done
      L=$O/${TAG}_ab_${libs//,/_}.json
      timeout -k 10 900 python -u tools/ab_libs.py --rounds 3 "${C[@]}" "${A[@]}" > $L 2>&1 || fail $step $? $L
      cat $L ;;
    stall:*)
      # SQ wave-state counters of one decode kernel per library build (tools/stall_profile.sh)
      IFS=: read -r _ libs cfg <<< "$step"
      timeout -k 10 900 bash tools/stall_profile.sh ${TAG}_$cfg "${CFG[$cfg]}" ${libs//,/ } > $O/${TAG}_stall_$cfg.log 2>&1 || fail $step $? $O/${TAG}_stall_$cfg.log
      tail -40 $O/${TAG}_stall_$cfg.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[$TAG] done"
