# PinSage aggregation / count_unique changes: tests, PinSage bench, DIEN graph-step kernel stats
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pinsage_gpu.py tests/test_embedding_gpu.py tests/test_pinsage_eval_gpu.py -q -x --timeout 400 --timeout-method thread > gpurun_out/c2_t.log 2>&1 || { tail -40 gpurun_out/c2_t.log; exit 1; }
tail -2 gpurun_out/c2_t.log
timeout -k 10 300 python benchmarks/bench_models.py --model pinsage --steps 20 --warmup 5 > gpurun_out/pin_b.json 2>gpurun_out/pin_b.err; tail -1 gpurun_out/pin_b.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dien2 -o run --output-format csv -- python benchmarks/bench_models.py --model dien --steps 10 --warmup 3 > gpurun_out/prof_dien2.log 2>&1 || { tail -20 gpurun_out/prof_dien2.log; exit 1; }
f=$(find gpurun_out/prof_dien2 -name "*kernel_stats.csv" | head -1)
python tools/summarize_prof.py "$f" gpurun_out/prof_dien2_summary.txt "dien graph step (rocprofv3 --kernel-trace --stats, bench_models --steps 10 --warmup 3)"
head -45 gpurun_out/prof_dien2_summary.txt | cut -c1-160
