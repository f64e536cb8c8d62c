# bench A/B of an environment toggle on one box (run under gpurun): VAR=RS_SORTED_GRAD bash tools/ab_env_bench.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in 1 0; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 100 --warmup 10 --cpu-baseline-steps 0 --pmc 0 \
      --compare-layerwise 0 --keras-line 0 > gpurun_out/abe_${v}_${r}.json 2> gpurun_out/abe.err || { tail -5 gpurun_out/abe.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abe_${v}_${r}.json').read().strip().splitlines()[-1]); print('$VAR', $v, 'run', $r, d['ms_per_step'], d['step_ms_distribution']['median'], {k: v['avg_us'] for k, v in d['roofline']['per_kernel'].items()}, d['roofline']['frac'])"
  done
done
