# secondary-model benchmarks (run under gpurun): MODELS="deepfm dlrm_cfg2" bash tools/models.sh
export TMPDIR=/tmp
for m in ${MODELS:-deepfm dlrm_cfg2 dien esmm mmoe pinsage eges}; do
  timeout -k 10 400 python benchmarks/bench_models.py --model $m ${MODEL_ARGS:-} > gpurun_out/m_$m.jsonl 2> gpurun_out/m_$m.err || { tail -20 gpurun_out/m_$m.err; exit 1; }
  cat gpurun_out/m_$m.jsonl
done
