# round-4 final: the whole GPU suite (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 600 --timeout-method thread > gpurun_out/r04_pytest_final.log 2>&1
rc=$?
tail -15 gpurun_out/r04_pytest_final.log
exit $rc
