# the update released by the train kernel (not the folds): parity, then the schedule A/B (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_step_gpu.py tests/test_northstar_gpu.py tests/test_chain_fwd_gpu.py -q -x --timeout 400 --timeout-method thread > gpurun_out/dep_t.log 2>&1 || { tail -30 gpurun_out/dep_t.log; exit 1; }
tail -1 gpurun_out/dep_t.log
REPS="1 2" VARIANTS="base afterfold graph2 graph2_afterfold" bash tools/step_ab.sh
