# round 4: sharded exchange tests + full-size configs + sort A/B (run under gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_sharded_gpu.py tests/test_esmm_gpu.py tests/test_fullsize_gpu.py tests/test_pinsage_gpu.py tests/test_embedding_gpu.py -v --timeout 600 --timeout-method thread > gpurun_out/r04_sh.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r04_sh.log | tail -50
timeout -k 10 120 python tools/sort_ab.py > gpurun_out/sort_ab.log 2>&1
tail -5 gpurun_out/sort_ab.log
exit $rc
