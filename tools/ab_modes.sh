# bench step modes side by side (run under gpurun): eager, one graph per step, one graph per pool
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for g in 0 1 2; do
    timeout -k 10 200 python bench.py --steps 100 --warmup 10 --cpu-baseline-steps 0 --pmc 0 \
      --compare-layerwise 0 --keras-line 0 --graph $g ${BENCH_ARGS:-} > gpurun_out/abm_${g}_${r}.json 2> gpurun_out/abm.err || { tail -5 gpurun_out/abm.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abm_${g}_${r}.json').read().strip().splitlines()[-1]); print('graph', $g, 'run', $r, d['ms_per_step'], d.get('step_ms_distribution', {}).get('median'))"
  done
done
