# round-6 session: A/B of this round's kernel steps (layered MS: HEAD -> layer bounds
# in registers -> + prefix-sum VN; BP: + prefix-sum column sums), then the parity files
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh r06d ab:head,lreg,msnew:msl2p10,msl2p05 ab:msnew,main:bpl2p10,bpf0 parity || exit 1
echo done
