# round 4: TunableOp over the GEMM shapes new this round (ESMM's shared first layer, MMOE's fused
# expert + gate block), on top of the committed table: entries already there are kept, the
# missing ones measured; the merged table is written back to gpurun_out/tune_new0.csv (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
cp recommender_amd/tuned/tunableop_mi355x.csv gpurun_out/tune_new0.csv
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune_new%d.csv
for m in esmm mmoe; do
  timeout -k 10 500 python benchmarks/bench_models.py --model $m --tuned-gemms 0 --steps 3 --warmup 2 > /dev/null 2> gpurun_out/tune_new_$m.err || { echo "$m failed"; tail -3 gpurun_out/tune_new_$m.err; exit 1; }
  echo "$m tuned: $(wc -l < gpurun_out/tune_new0.csv) lines"
done
