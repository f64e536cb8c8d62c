export TMPDIR=/tmp
: > gpurun_out/models.jsonl
for m in deepfm dien esmm mmoe pinsage eges; do
  timeout -k 10 300 python benchmarks/bench_models.py --model $m >> gpurun_out/models.jsonl 2> gpurun_out/models_$m.err || { echo "$m failed"; tail -5 gpurun_out/models_$m.err; exit 1; }
done
cut -c1-300 gpurun_out/models.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dien -o run --output-format csv -- python benchmarks/bench_models.py --model dien --steps 10 --warmup 3 > gpurun_out/prof_dien.log 2>&1 || { echo prof failed; exit 1; }
echo prof ok
