bash scripts/gpu_sessions.sh && bash scripts/pmc_cmd.sh cfg5 mxstream.models.bench_configs --config 5 --steps 3 --warmup 8
