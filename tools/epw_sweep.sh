timeout -k 10 300 python -m pytest tests/test_interaction_gpu.py tests/test_sharded_gpu.py -x -q > gpurun_out/t_pipe.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/t_pipe.log; exit 1; }
tail -1 gpurun_out/t_pipe.log
for e in 16; do
  RS_INTER_BWD_EPW=$e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 --pmc 0 > gpurun_out/epw_$e.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/epw_$e.log').read().strip().splitlines()[-1]);print('epw $e', d['ms_per_step'], d['kernels']['rs_dlrm_interaction_bwd']['avg_us'], d['kernels']['rs_dlrm_interaction_fwd']['avg_us'])"
done
