# A/B of variant builds (python -m recommender_amd.build --variant NAME -DFLAGS...) on one box:
# VARIANTS="a b" bash tools/ab_variants.sh — per library: the isolated path (ONLY=...) and, with
# STEP=1, a short bench.py step time; two rounds
export TMPDIR=/tmp
for rep in 1 2; do
for v in base ${VARIANTS}; do
  if [ $v = base ]; then unset RS_LIB; else export RS_LIB=recommender_amd/_lib/variants/$v.so; fi
  timeout -k 10 200 python benchmarks/bench_kernels.py --only ${ONLY:-dlrm_path} > gpurun_out/abv_$v.jsonl 2> gpurun_out/abv_$v.err || { tail -20 gpurun_out/abv_$v.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/abv_$v.jsonl'):
    if l.startswith('{'):
        d=json.loads(l)
        if '${FILTER:-}' in d['kernel']: print('$v'.ljust(10), f\"{d['avg_us']:8.1f}\", d['kernel'][:70])"
  if [ "${STEP:-0}" = 1 ]; then
    timeout -k 10 300 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 --steps 30 > gpurun_out/abv_b_$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/abv_b_$v.json').read().strip().splitlines()[-1]);print('$v'.ljust(10),'step ms',d['ms_per_step'])"
  fi
done
done
