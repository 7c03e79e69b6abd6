# round-6 session: A/B of the AMDGPU machine-scheduler strategies (max-ilp,
# max-memory-clause, iterative-minreg; iterative-ilp crashes the compiler on osd_kernels.hip) against the default, every decoder
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06p ab:main,silp,smem,sitmr:msl2p10,bpl2p10,bpf0,head osdab:main,silp,smem,sitmr || exit 1
echo done
