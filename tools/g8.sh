export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_mlp_chain_gpu.py tests/test_interaction_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mlp.log 2>&1 || { tail -40 gpurun_out/mlp.log; exit 1; }
tail -1 gpurun_out/mlp.log
timeout -k 10 300 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 > gpurun_out/bench_g0.log 2>&1 || { tail -20 gpurun_out/bench_g0.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_g0.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 --pmc 0 --compare-layerwise 0 > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof failed"; exit 1; }
grep -i "chain_reduce\|fold_" gpurun_out/prof_bench/run_kernel_stats.csv | cut -d, -f1-6
