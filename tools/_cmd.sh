TESTS="tests/test_fused_step_gpu.py tests/test_northstar_gpu.py" TLIM=600 bash tools/gpu_tests.sh && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" && bash tools/bench_quick.sh
