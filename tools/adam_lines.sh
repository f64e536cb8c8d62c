# north-star secondary lines with the reference's active optimizer (run under gpurun)
export TMPDIR=/tmp
for o in lazy_adam keras_adam; do
  timeout -k 10 300 python bench.py --optimizer $o --steps 10 --warmup 3 --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 > gpurun_out/adam_$o.json 2> gpurun_out/adam_$o.err || { tail -20 gpurun_out/adam_$o.err; exit 1; }
  tail -1 gpurun_out/adam_$o.json | cut -c1-400
done
timeout -k 10 300 python benchmarks/bench_models.py --model dlrm_cfg2 --optimizer keras_adam > gpurun_out/m_dlrm_cfg2_adam.jsonl 2> gpurun_out/m_cfg2a.err || { tail -20 gpurun_out/m_cfg2a.err; exit 1; }
cat gpurun_out/m_dlrm_cfg2_adam.jsonl
