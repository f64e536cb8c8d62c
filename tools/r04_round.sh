# round-4 final check (run under gpurun): the whole GPU suite, the default bench line (with PMC
# passes) and an isolated kernel trace of the id sort (tools/sort_ab.py)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 6 --timeout 500 --timeout-method thread > gpurun_out/r04_pytest.log 2>&1
rc=$?
tail -12 gpurun_out/r04_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r04_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r04_bench.log; exit 1; }
tail -1 gpurun_out/r04_bench.log > gpurun_out/r04_bench.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sort_kt -o run --output-format csv -- python tools/sort_ab.py --iters 50 > gpurun_out/sort_kt.log 2>&1 || { tail -20 gpurun_out/sort_kt.log; exit 1; }
exit $rc
