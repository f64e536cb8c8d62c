# sort launches with a capped grid (tile loop): bit-exact tests at a tiny cap, then the step A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
RS_SORT_BLOCKS=7 timeout -k 10 600 python -u -m pytest tests/test_embedding_gpu.py -q -x -k "sort or dedup or apply or golden" --timeout 400 --timeout-method thread > gpurun_out/sg_t.log 2>&1 || { tail -30 gpurun_out/sg_t.log; exit 1; }
tail -1 gpurun_out/sg_t.log
REPS="1 2" VARIANTS="base sb128 sb64 pf_sb64 pf_sb32" bash tools/step_ab.sh
