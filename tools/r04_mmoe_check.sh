# round-4: fused MMOE block + ESMM shared first layer: unit tests, cfg4 full-size oracle checks,
# then the three multitask lines and a kernel trace of MMOE (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_esmm_gpu.py \
  "tests/test_fullsize_gpu.py::test_cfg4_full_size_keras_adam_steps_vs_oracle" > gpurun_out/r04_mmoe_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_mmoe_tests.log; [ $rc -eq 0 ] || exit $rc
for m in mmoe esmm; do
  timeout -k 10 300 python benchmarks/bench_models.py --model $m 2>gpurun_out/models_$m.err | tail -1 | cut -c1-200 || exit 1
done
timeout -k 10 300 python tools/op_census.py --model mmoe > gpurun_out/op_census_mmoe2.txt 2>&1 && tail -1 gpurun_out/op_census_mmoe2.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_mmoe -o run -- python $GRAFT_REPO_ROOT/benchmarks/bench_models.py --model mmoe --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_mmoe.log 2>&1; echo prof rc $?
