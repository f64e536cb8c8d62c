# round-4 check: full GPU suite, default bench line, self-launched world-2 gloo bench (run under gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r04_pytest.log; exit 1; }
tail -3 gpurun_out/r04_pytest.log
timeout -k 10 600 python bench.py > gpurun_out/r04_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r04_bench.log; exit 1; }
tail -1 gpurun_out/r04_bench.log > gpurun_out/r04_bench.json
RS_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --pmc 0 --steps 5 --warmup 2 --compare-layerwise 0 --weak-secondary 0 > gpurun_out/r04_w2.log 2>&1 || { echo "w2 failed"; tail -30 gpurun_out/r04_w2.log; exit 1; }
tail -1 gpurun_out/r04_w2.log | cut -c1-400
echo done
