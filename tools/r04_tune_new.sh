# round 4: TunableOp over the GEMM shapes new this round (ESMM's shared first layer, MMOE's fused
# expert + gate block), on top of the committed table: its entries are kept, the missing shapes
# measured; the merged table lands in gpurun_out/tune_new0.csv, then the two models are benched
# with it (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
cp recommender_amd/tuned/tunableop_mi355x.csv gpurun_out/tune_new0.csv
for m in esmm mmoe; do
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune_new%d.csv \
  PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 \
    timeout -k 10 400 python benchmarks/bench_models.py --model $m --tuned-gemms 0 --steps 2 --warmup 1 > /dev/null 2> gpurun_out/tune_new_$m.err || { echo "$m failed"; tail -3 gpurun_out/tune_new_$m.err; exit 1; }
  echo "$m tuned: $(wc -l < gpurun_out/tune_new0.csv) lines"
done
cp gpurun_out/tune_new0.csv recommender_amd/tuned/tunableop_mi355x.csv
for m in mmoe esmm; do
  timeout -k 10 300 python benchmarks/bench_models.py --model $m 2>gpurun_out/models_$m.err | tail -1 | cut -c1-400 || exit 1
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_mmoe2 -o run -- python $GRAFT_REPO_ROOT/benchmarks/bench_models.py --model mmoe --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_mmoe2.log 2>&1; echo prof rc $?
