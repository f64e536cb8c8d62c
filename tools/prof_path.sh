# isolated embedding-path launches + their rocprof summary (run under gpurun)
export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/bench_kernels.py --only dlrm_path > gpurun_out/path.jsonl 2> gpurun_out/path.err || { tail -20 gpurun_out/path.err; exit 1; }
cat gpurun_out/path.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_path -o run --output-format csv -- python benchmarks/bench_kernels.py --only dlrm_path --iters 10 > gpurun_out/prof_path.log 2>&1 || { tail -5 gpurun_out/prof_path.log; exit 1; }
python tools/summarize_prof.py gpurun_out/prof_path/run_kernel_stats.csv gpurun_out/prof_path_summary.txt "isolated path" && head -20 gpurun_out/prof_path_summary.txt
