set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab_env.py QLDPC_NO_LAYERED_FAST LP118_0 MS L None 50 262144 3 > gpurun_out/abenv.jsonl 2>gpurun_out/abenv.err || exit $?
timeout -k 10 600 python tools/ab_env.py QLDPC_NO_LAYERED_FAST LP118_2 MS L 0.05 50 262144 3 >> gpurun_out/abenv.jsonl 2>>gpurun_out/abenv.err
