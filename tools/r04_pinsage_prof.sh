# round 4: PinSage step after the fused loss / genre lookup — bench lines and the kernel profile
# of the graph step (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pinsage_gpu.py -k "margin or multihot or graph" > gpurun_out/r04_pinsage_tests2.log 2>&1
rc=$?; tail -1 gpurun_out/r04_pinsage_tests2.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python benchmarks/bench_models.py --model pinsage 2>/dev/null | tail -1 | cut -c1-100 || exit 1
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_pinsage2 -o run -- python $GRAFT_REPO_ROOT/benchmarks/bench_models.py --model pinsage --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_pinsage2.log 2>&1; echo prof rc $?
