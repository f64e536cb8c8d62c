export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_mlp_chain_gpu.py tests/test_interaction_gpu.py tests/test_embedding_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mlp.log 2>&1 || { tail -40 gpurun_out/mlp.log; exit 1; }
tail -1 gpurun_out/mlp.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 > gpurun_out/bench_g0.log 2>&1 || { tail -20 gpurun_out/bench_g0.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_g0.log
