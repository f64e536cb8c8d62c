# targeted GPU tests + short bench (run under gpurun)
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_chain_fwd_gpu.py tests/test_mlp_chain_gpu.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/qc_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/qc_pytest.log; exit 1; }
tail -1 gpurun_out/qc_pytest.log
timeout -k 10 300 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 --steps 40 > gpurun_out/qc_bench.json 2> gpurun_out/qc_bench.err || { tail -20 gpurun_out/qc_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/qc_bench.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['value'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
