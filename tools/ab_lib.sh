# A/B of the built library against librecsys_hip_base.so on one box (run under gpurun):
# parity tests of the sparse path first, then the isolated north-star path, alternating
export TMPDIR=/tmp
L=recommender_amd/_lib
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_embedding_gpu.py tests/test_sharded_gpu.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -1 gpurun_out/ab_pytest.log
cp $L/librecsys_hip.so /tmp/new.so; cp $L/librecsys_hip_base.so /tmp/base.so
for v in new base new base; do
  cp /tmp/$v.so $L/librecsys_hip.so
  timeout -k 10 200 python benchmarks/bench_kernels.py --only dlrm_path > gpurun_out/ab_$v.jsonl 2> gpurun_out/ab_$v.err || { tail -20 gpurun_out/ab_$v.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/ab_$v.jsonl'):
    if l.startswith('{'):
        d=json.loads(l)
        if 'apply' in d['kernel'] or 'path' in d['kernel']: print('$v', d['kernel'][:40], d['avg_us'])"
done
cp /tmp/new.so $L/librecsys_hip.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_prof -o run --output-format csv -- python benchmarks/bench_kernels.py --only dlrm_path --iters 10 > gpurun_out/ab_prof.log 2>&1 || { tail -5 gpurun_out/ab_prof.log; exit 1; }
grep -E "seg_" gpurun_out/ab_prof/run_kernel_stats.csv | cut -c1-200
