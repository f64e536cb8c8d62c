# DIEN parity + graph-step bench (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dien_gpu.py tests/test_dien_step_gpu.py "tests/test_fullsize_gpu.py::test_cfg3_dien_full_size_step_vs_oracle" -q -x --timeout 400 --timeout-method thread > gpurun_out/dien_t.log 2>&1 || { tail -40 gpurun_out/dien_t.log; exit 1; }
tail -2 gpurun_out/dien_t.log
for i in 1 2; do timeout -k 10 300 python benchmarks/bench_models.py --model dien --steps 30 --warmup 3 2>/dev/null | tail -1 | cut -c1-200; done
