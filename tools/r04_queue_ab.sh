# round 4: the apply walk with queued table updates (RS_APPLY_QUEUE=1) — parity tests with it on,
# then interleaved bench A/B (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
RS_APPLY_QUEUE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_northstar_gpu.py tests/test_fused_step_gpu.py tests/test_embedding_gpu.py > gpurun_out/q_tests.log 2>&1
rc=$?; tail -2 gpurun_out/q_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  RS_APPLY_QUEUE=$v timeout -k 10 300 python bench.py --steps 200 --warmup 20 --pmc 0 --cpu-baseline-steps 0 > gpurun_out/q_bench_$v.json 2> gpurun_out/q_bench_$v.err || exit 1
  python - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/q_bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
pk = d["roofline"]["per_kernel"]
print("queue", sys.argv[1], "ms", d["ms_per_step"], "apply alone", pk["rs_embedding_apply_scaled"]["avg_us"],
      "in step", pk["rs_embedding_apply_scaled"]["in_step_span_us"], "frac", d["roofline"]["frac"])
PY
done
