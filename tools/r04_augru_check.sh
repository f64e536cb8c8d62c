# round 4: the AUGRU forward back to its one-step-at-a-time form — DIEN tests, bench, kernel profile (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_dien_gpu.py tests/test_dien_step_gpu.py "tests/test_fullsize_gpu.py::test_cfg3_dien_full_size_step_vs_oracle" > gpurun_out/r04_augru_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04_augru_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python benchmarks/bench_models.py --model dien 2>/dev/null | tail -1 | cut -c1-90 || exit 1; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_dien_late2 -o run -- python $GRAFT_REPO_ROOT/benchmarks/bench_models.py --model dien --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_dien_late2.log 2>&1; echo prof rc $?
