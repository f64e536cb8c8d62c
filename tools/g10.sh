export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python benchmarks/bench_models.py --model deepfm > gpurun_out/deepfm.jsonl 2>/dev/null || exit 1
cut -c1-200 gpurun_out/deepfm.jsonl
timeout -k 10 300 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 > gpurun_out/bench_g0.log 2>&1 || { tail -20 gpurun_out/bench_g0.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_g0.log
