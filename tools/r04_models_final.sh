# round-4 final model lines (gpurun): one bench_models line per configuration into one jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r04_models_bench.jsonl
for m in deepfm deepfm_file dlrm_cfg2 dien esmm mmoe pinsage eges; do
  timeout -k 10 400 python benchmarks/bench_models.py --model $m 2>gpurun_out/models_$m.err | tail -1 >> gpurun_out/r04_models_bench.jsonl || { echo "$m failed"; tail -5 gpurun_out/models_$m.err; }
  tail -1 gpurun_out/r04_models_bench.jsonl | cut -c1-160
done
