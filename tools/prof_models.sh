export TMPDIR=/tmp
for m in dien pinsage mmoe eges; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$m -o run --output-format csv -- python benchmarks/bench_models.py --model $m --steps 10 --warmup 3 > gpurun_out/prof_$m.log 2>&1 || { echo "$m failed rc=$?"; exit 1; }
  echo "$m ok"; tail -1 gpurun_out/prof_$m.log
done
