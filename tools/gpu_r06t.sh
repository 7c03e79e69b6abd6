# round-6 session: A/B of machine-scheduler tuning flags (AMDGPU register-pressure trackers,
# occupancy/latency metric bias 0 / 100, memory-op clustering off) on the headline, layered MS
# and layered BP kernels; the OSD engine's slot reads batched (main) against HEAD (h7) and the
# flag builds; the OSD parity file on main
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06t osdab:main,h7,t1,t2,t3,t4 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_osd.py tests/test_gpu_simulator.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r06t_parity_osd.log 2>&1; tail -2 gpurun_out/r06t_parity_osd.log
bash tools/gpu_run.sh r06t ab:h7,t1,t2,t3,t4:head,msl2p10,bpl2p10 || exit 1
echo done
