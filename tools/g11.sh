export TMPDIR=/tmp
: > gpurun_out/models.jsonl
for m in deepfm dien esmm mmoe pinsage eges; do
  timeout -k 10 300 python benchmarks/bench_models.py --model $m >> gpurun_out/models.jsonl 2> gpurun_out/models_$m.err || { echo "$m failed"; tail -5 gpurun_out/models_$m.err; exit 1; }
done
cut -c1-110 gpurun_out/models.jsonl
for t in 1 0; do
timeout -k 10 300 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 --tuned-gemms $t > gpurun_out/bench_t$t.log 2>&1 || { tail -20 gpurun_out/bench_t$t.log; exit 1; }
echo tuned=$t; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_t$t.log
done
