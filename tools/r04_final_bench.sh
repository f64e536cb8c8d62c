# round-4 final measurements (gpurun): the default bench line (PMC passes included), the kernel
# stats of the same step under rocprofv3, the train kernel's SQ counters
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r04_bench_final.log 2>&1 || { tail -30 gpurun_out/r04_bench_final.log; exit 1; }
tail -1 gpurun_out/r04_bench_final.log > gpurun_out/r04_bench_final.json
python -c "import json; d=json.load(open('gpurun_out/r04_bench_final.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], {k: v['avg_us'] for k, v in d['roofline']['per_kernel'].items()}, d.get('keras_adam', {}).get('value'), d['cpu_baseline'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_final -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --pmc 0 --keras-line 0 --weak-secondary 0 --compare-layerwise 0 --cpu-baseline-steps 0 > gpurun_out/prof_bench_final.log 2>&1 || { tail -20 gpurun_out/prof_bench_final.log; exit 1; }
f=$(find gpurun_out/prof_bench_final -name "*kernel_stats.csv" | head -1)
python tools/summarize_prof.py "$f" gpurun_out/prof_bench_final_summary.txt "rocprofv3 --kernel-trace --stats -- python bench.py --steps 20 --warmup 5 --pmc 0 (round 4 final tree)"
head -14 gpurun_out/prof_bench_final_summary.txt | cut -c1-150
bash tools/pmc_train.sh > gpurun_out/r04_train_pmc.txt 2>&1; cat gpurun_out/r04_train_pmc.txt
