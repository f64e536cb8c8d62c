export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "tests/test_fullsize_gpu.py::test_cfg4_full_size_keras_adam_steps_vs_oracle" "tests/test_fullsize_gpu.py::test_cfg5_ml20m_model_step_vs_float64" "tests/test_pinsage_gpu.py::test_world2_pinsage_static_step_and_missing_gradients" tests/test_train_unit_gpu.py -v --timeout 500 --timeout-method thread > gpurun_out/r04_fix.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r04_fix.log | tail -20
timeout -k 10 120 python tools/sort_ab.py > gpurun_out/sort_ab.log 2>&1; tail -4 gpurun_out/sort_ab.log
timeout -k 10 300 python benchmarks/bench_models.py --model deepfm_file > gpurun_out/cfg1_file.json 2> gpurun_out/cfg1_file.err; tail -2 gpurun_out/cfg1_file.json; tail -3 gpurun_out/cfg1_file.err

VARIANTS="ss us ssus nosb stag2 prio" ONLY=dlrm_path FILTER=train timeout -k 10 600 bash tools/ab_variants.sh > gpurun_out/ab_train.txt 2>&1; cat gpurun_out/ab_train.txt | tail -12
exit $rc
