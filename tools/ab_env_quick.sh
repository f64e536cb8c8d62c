# interleaved A/B of environment settings on one box (run under gpurun):
# AB_ENVS="RS_X=0 RS_X=1" REPS=3 BENCH_ARGS="..." bash tools/ab_env_quick.sh
export TMPDIR=/tmp
for rep in $(seq ${REPS:-3}); do
for e in ${AB_ENVS}; do
  env $e timeout -k 10 300 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 --keras-line 0 --steps ${STEPS:-60} ${BENCH_ARGS:-} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);q=d.get('step_ms_distribution') or {};print('$e'.ljust(24),'ms/step',d['ms_per_step'],'median',q.get('median'),'p90',q.get('p90'))"
done
done
