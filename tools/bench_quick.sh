# short bench (run under gpurun): no PMC passes, no CPU baseline, no layerwise comparison
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 --steps ${STEPS:-30} ${BENCH_ARGS:-} > gpurun_out/qb.json 2> gpurun_out/qb.err || { tail -20 gpurun_out/qb.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/qb.json').read().strip().splitlines()[-1])
r=d['roofline'];print('ms/step',d['ms_per_step'],'value',d['value'],'path frac',r['frac'],'path us',r['us_per_step'])
for k,v in r['per_kernel'].items(): print('  ',k,v['avg_us'],v['frac'],'in-step',v['in_step_span_us'])"
