# one eager MMOE step as a kernel sequence with grid sizes (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/mmoe_kt -o run --output-format csv -- python benchmarks/bench_models.py --model mmoe --steps 4 --warmup 2 > gpurun_out/mmoe_kt.log 2>&1 || { tail -20 gpurun_out/mmoe_kt.log; exit 1; }
f=$(find gpurun_out/mmoe_kt -name "*kernel_trace.csv" | head -1)
python tools/step_trace.py "$f" --marker "radix_hist_kernel<9, true" > gpurun_out/mmoe_step_trace.txt; head -3 gpurun_out/mmoe_step_trace.txt
