bash tools/gpu_counters_cfg.sh bpF LP118_0 BP F 0.05 100 262144 && bash tools/gpu_counters_cfg.sh bpL LP118_2 BP L 0.1 100 65536
