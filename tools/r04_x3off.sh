# the linear layers' fused activations with the library GEMMs (RS_GEMM_X3 off): model parity (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_esmm_gpu.py tests/test_deepfm_gpu.py tests/test_mlp_chain_gpu.py "tests/test_fullsize_gpu.py::test_cfg4_full_size_keras_adam_steps_vs_oracle" tests/test_sharded_gpu.py -q --maxfail 5 --timeout 600 --timeout-method thread > gpurun_out/x3off_t.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error:|max err" gpurun_out/x3off_t.log | head -20
[ $rc -eq 0 ] || exit $rc
for m in esmm mmoe; do timeout -k 10 300 python benchmarks/bench_models.py --model $m --steps 20 --warmup 3 2>/dev/null | tail -1 | cut -c1-160; done
