# round-4: segmented densify test + DIEN step parity, then the torch-glue census of DIEN / ESMM / MMOE (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_embedding_gpu.py tests/test_dien_step_gpu.py tests/test_esmm_gpu.py -k "densify or concat or dien or esmm or shared" > gpurun_out/r04_census_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_census_tests.log; [ $rc -eq 0 ] || exit $rc
for m in dien mmoe esmm; do
  timeout -k 10 300 python tools/op_census.py --model $m > gpurun_out/op_census_$m.txt 2>&1 || { tail -5 gpurun_out/op_census_$m.txt; exit 1; }
  tail -1 gpurun_out/op_census_$m.txt
done
