# A/B of the bench step with and without the next batch's sort launched after the train kernel
# (bench.py --prefetch 1), alternating, 2 runs each (run under gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for p in 0 1; do
    timeout -k 10 200 python bench.py --steps 100 --warmup 10 --cpu-baseline-steps 0 --pmc 0 \
      --compare-layerwise 0 --keras-line 0 --prefetch $p > gpurun_out/abp_${p}_${r}.json 2> gpurun_out/abp.err || { tail -5 gpurun_out/abp.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/abp_${p}_${r}.json').read().strip().splitlines()[-1]); print('prefetch', $p, 'run', $r, d['ms_per_step'], d['step_ms_distribution']['median'], d['roofline']['per_kernel']['rs_sort_ids']['avg_us'])"
  done
done
