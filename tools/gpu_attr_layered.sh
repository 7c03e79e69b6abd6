set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/attr.jsonl
V="base:QLDPC_LIB=qldpcsim_amd/_build/var_base.so nocn:QLDPC_LIB=qldpcsim_amd/_build/var_nocn.so novn:QLDPC_LIB=qldpcsim_amd/_build/var_novn.so noflip:QLDPC_LIB=qldpcsim_amd/_build/var_noflip.so nostop:QLDPC_LIB=qldpcsim_amd/_build/var_nostop.so"
for cfg in "LP118_2 MS L None 50 65536" "LP118_0 MS L None 50 65536"; do
  echo "$cfg" >> gpurun_out/attr.jsonl
  timeout -k 10 300 python tools/ab_variants.py $cfg 2 $V >> gpurun_out/attr.jsonl 2>> gpurun_out/attr.err || exit $?
done
