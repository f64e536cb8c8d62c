TESTS="tests/test_embedding_gpu.py tests/test_fused_step_gpu.py" TLIM=400 bash tools/gpu_tests.sh && STEP=1 FILTER="apply_scaled (alone)" VARIANTS="t32single not32" bash tools/ab_variants.sh
