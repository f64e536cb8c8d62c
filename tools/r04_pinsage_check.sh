# round 4: fused PinSage pair scores + margin loss — PinSage tests (cfg5 full size incl.), the
# bench line and the glue census (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_pinsage_gpu.py \
  "tests/test_fullsize_gpu.py::test_cfg5_ml20m_model_step_vs_float64" > gpurun_out/r04_pinsage_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_pinsage_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python benchmarks/bench_models.py --model pinsage 2>/dev/null | tail -1 | cut -c1-120 || exit 1
done
timeout -k 10 300 python tools/op_census.py --model pinsage > gpurun_out/op_census_pinsage2.txt 2>&1 && tail -1 gpurun_out/op_census_pinsage2.txt
