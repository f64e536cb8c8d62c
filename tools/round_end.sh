# round-end refresh: full bench line (with PMC traffic + cpu baseline), rocprof kernel stats
# of the bench, and the isolated north-star path (run under gpurun)
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log > gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 --pmc 0 --compare-layerwise 0 --keras-line 0 > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof failed"; exit 1; }
timeout -k 10 300 python benchmarks/bench_kernels.py --only dlrm_path > gpurun_out/path.jsonl 2> gpurun_out/path.err || { tail -20 gpurun_out/path.err; exit 1; }
cat gpurun_out/path.jsonl
echo done
