# relu in the library GEMM epilogue: parity + A/B (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_esmm_gpu.py tests/test_deepfm_gpu.py tests/test_mlp_chain_gpu.py tests/test_dien_step_gpu.py "tests/test_fullsize_gpu.py::test_cfg4_full_size_keras_adam_steps_vs_oracle" -q --maxfail 3 --timeout 600 --timeout-method thread > gpurun_out/relu_t.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|max err" gpurun_out/relu_t.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for m in esmm mmoe; do for e in 1 0; do RS_RELU_EPILOGUE=$e timeout -k 10 300 python benchmarks/bench_models.py --model $m --steps 20 --warmup 3 2>/dev/null | tail -1 | cut -c1-120 | sed "s/^/relu_epi=$e /"; done; done
