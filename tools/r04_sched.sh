# main-stream update schedule + DIEN fused nodes: parity tests, then the schedule A/B (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_step_gpu.py tests/test_northstar_gpu.py tests/test_dien_gpu.py tests/test_dien_step_gpu.py "tests/test_embedding_gpu.py::test_concat_lookup_matches_cat_of_lookups" tests/test_chain_fwd_gpu.py -q -x --timeout 400 --timeout-method thread > gpurun_out/sched_t.log 2>&1 || { tail -40 gpurun_out/sched_t.log; exit 1; }
tail -2 gpurun_out/sched_t.log
bash tools/step_ab.sh
timeout -k 10 300 python benchmarks/bench_models.py --model dien --steps 20 --warmup 3 > gpurun_out/dien_b.json 2>gpurun_out/dien_b.err; tail -1 gpurun_out/dien_b.json | cut -c1-300
