# PyTorch TunableOp over the dense GEMM shapes of every benchmarked model; the merged results
# file is committed as recommender_amd/tuned/tunableop_mi355x.csv
export TMPDIR=/tmp
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune_all%d.csv
for m in dien mmoe esmm pinsage eges deepfm; do
  timeout -k 10 600 python benchmarks/bench_models.py --model $m --steps 3 --warmup 2 > /dev/null 2> gpurun_out/tune_$m.err || { echo "$m failed"; tail -3 gpurun_out/tune_$m.err; exit 1; }
  echo "$m tuned: $(wc -l < gpurun_out/tune_all0.csv) lines"
done
timeout -k 10 600 python bench.py --steps 3 --warmup 2 --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 1 > /dev/null 2> gpurun_out/tune_dlrm.err || { echo dlrm failed; exit 1; }
echo "dlrm tuned: $(wc -l < gpurun_out/tune_all0.csv) lines"
