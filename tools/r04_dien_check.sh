# round-4: DIEN glue cuts (uint8 mask once, shared valid-row lists, BatchNormalization kernels):
# DIEN tests incl. the cfg3 full-size oracle step, then the bench line and the glue census (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_dien_gpu.py \
  tests/test_dien_step_gpu.py tests/test_dien_proj_gpu.py "tests/test_fullsize_gpu.py::test_cfg3_dien_full_size_step_vs_oracle" \
  > gpurun_out/r04_dien_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_dien_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/bench_models.py --model dien 2>gpurun_out/models_dien.err | tail -1 | cut -c1-200 || exit 1
timeout -k 10 300 python tools/op_census.py --model dien > gpurun_out/op_census_dien2.txt 2>&1 && tail -1 gpurun_out/op_census_dien2.txt
timeout -k 10 300 python tools/op_census.py --model pinsage > gpurun_out/op_census_pinsage.txt 2>&1 && tail -1 gpurun_out/op_census_pinsage.txt
