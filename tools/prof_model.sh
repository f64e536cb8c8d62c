# rocprof kernel summary of one secondary model's bench (run under gpurun): MODEL=dien bash tools/prof_model.sh
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$MODEL -o run --output-format csv -- python benchmarks/bench_models.py --model $MODEL --steps 10 --warmup 3 > gpurun_out/prof_$MODEL.log 2>&1 || { tail -5 gpurun_out/prof_$MODEL.log; exit 1; }
python tools/summarize_prof.py gpurun_out/prof_$MODEL/run_kernel_stats.csv gpurun_out/prof_${MODEL}_summary.txt "$MODEL" && head -40 gpurun_out/prof_${MODEL}_summary.txt
tail -1 gpurun_out/prof_$MODEL.log
