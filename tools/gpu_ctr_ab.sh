bash tools/gpu_counters.sh v2 QLDPC_FLOOD_V2=1 && bash tools/gpu_counters.sh compact
