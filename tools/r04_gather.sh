# flat float2 gather for 18-wide rows: parity + cfg4 benches (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_embedding_gpu.py tests/test_esmm_gpu.py "tests/test_fullsize_gpu.py::test_cfg4_full_size_keras_adam_steps_vs_oracle" -q -x --timeout 600 --timeout-method thread > gpurun_out/gather_t.log 2>&1 || { tail -30 gpurun_out/gather_t.log; exit 1; }
tail -1 gpurun_out/gather_t.log
for m in esmm mmoe; do timeout -k 10 300 python benchmarks/bench_models.py --model $m --steps 20 --warmup 3 2>/dev/null | tail -1 | cut -c1-250; done
