# kernel-trace timeline of the DLRM bench step (run under gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl -o run --output-format csv -- python bench.py --steps 8 --warmup 3 --cpu-baseline-steps 0 --pmc 0 --compare-layerwise 0 --graph ${GRAPH:-0} ${BENCH_ARGS:-} > gpurun_out/tl.log 2>&1 || { tail -5 gpurun_out/tl.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/tl.log
f=$(find gpurun_out/tl -name "*kernel_trace.csv" | head -1)
python tools/step_timeline.py $f ${MARK:-dlrm_train_pipe}
