# Build A/B library variants of the HIP decoder into qldpcsim_amd/_build/var_<name>.so
# usage: bash tools/build_variants.sh name1 "EXTRA FLAGS" [name2 "FLAGS" ...]
#        name "HEAD" as flags builds the committed sources (git HEAD) instead.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  if [ "$flags" = "HEAD" ]; then
    tmp=$(mktemp -d)
    (cd "$ROOT" && git archive HEAD qldpcsim_amd/csrc include) | tar -x -C "$tmp"
    rm -f "$ROOT/qldpcsim_amd/_build/var_$name.so"   # archived sources carry old mtimes: make would skip
    make -s -C "$tmp/qldpcsim_amd/csrc" OUT_DIR="$ROOT/qldpcsim_amd/_build" LIB=var_$name.so 2>&1 | grep -i error || true
    rm -rf "$tmp"
  else
    touch "$ROOT/qldpcsim_amd/csrc/decoder_kernels.hip"
    make -s -C "$ROOT/qldpcsim_amd/csrc" LIB=var_$name.so EXTRA="-DQLDPC_EXPERIMENTS $flags" 2>&1 | grep -i error || true
  fi
  ls -la "$ROOT/qldpcsim_amd/_build/var_$name.so"
done
