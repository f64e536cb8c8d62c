# PinSage: parity tests + the bench in each mode (run under gpurun): MODES="static graph"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pinsage_gpu.py ${EXTRA_TESTS:-} -x -q --timeout 120 --timeout-method thread > gpurun_out/pin_tests.log 2>&1 || { tail -60 gpurun_out/pin_tests.log; exit 1; }
tail -3 gpurun_out/pin_tests.log
for m in ${MODES:-dynamic static graph}; do
  timeout -k 10 200 python benchmarks/bench_models.py --model pinsage --pinsage-mode $m > gpurun_out/pin_$m.json 2> gpurun_out/pin_$m.err || { tail -30 gpurun_out/pin_$m.err; exit 1; }
  cut -c1-200 gpurun_out/pin_$m.json
done
