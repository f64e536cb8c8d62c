export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log > gpurun_out/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 --pmc 0 --compare-layerwise 0 > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof failed"; exit 1; }
for m in pinsage eges; do
  timeout -k 10 300 python benchmarks/bench_models.py --model $m > gpurun_out/m_$m.jsonl 2>/dev/null || exit 1
done
echo done
