# round-4 secondary-config profiles (run under gpurun): rocprof kernel stats of DIEN (graph), ESMM
# and MMOE at cfg3 / cfg4 sizes, and their bench lines
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in dien esmm mmoe; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$m -o run --output-format csv -- python benchmarks/bench_models.py --model $m --steps 10 --warmup 3 > gpurun_out/prof_$m.log 2>&1 || { tail -20 gpurun_out/prof_$m.log; exit 1; }
  f=$(find gpurun_out/prof_$m -name "*kernel_stats.csv" | head -1)
  python tools/summarize_prof.py "$f" gpurun_out/prof_${m}_summary.txt "$m (rocprofv3 --kernel-trace --stats, bench_models --steps 10 --warmup 3)"
  head -25 gpurun_out/prof_${m}_summary.txt
  grep '^{' gpurun_out/prof_$m.log | tail -1 | cut -c1-300
done
