# targeted GPU tests (run under gpurun): TESTS="tests/x.py ..." bash tools/gpu_tests.sh
export TMPDIR=/tmp
timeout -k 10 ${TLIM:-900} python -u -m pytest ${TESTS:-tests -m gpu} -x -v -s --timeout 600 --timeout-method thread > gpurun_out/gt_pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/gt_pytest.log; exit 1; }
grep -E "passed|failed|step [0-9]|smoke ok" gpurun_out/gt_pytest.log | tail -20
