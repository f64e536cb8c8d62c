export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 --pmc 0 --compare-layerwise 0 > gpurun_out/prof_q.log 2>&1 || { echo "rocprof failed"; tail gpurun_out/prof_q.log; exit 1; }
tail -1 gpurun_out/prof_q.log | cut -c1-300
