# round-6 session: full GPU suite at the new kernels, counter profiles of the kernels
# whose machine code changed (layered MS, layered BP), OSD write attribution
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06e tests roof-msl roof-bp || exit 1
for l in main osdwpe3; do
  [ $l = main ] && P=qldpcsim_amd/_build/libqldpc_hip.so || P=qldpcsim_amd/_build/var_$l.so
  QLDPC_LIB=$P bash tools/gpu_profile_program.sh r06e_osd_$l tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 2 || exit 1
done
echo done
