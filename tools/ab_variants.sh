# A/B of variant builds (python -m recommender_amd.build --variant NAME -DFLAGS...) on one box:
# VARIANTS="a b" bash tools/ab_variants.sh  — the isolated north-star path per library, twice
export TMPDIR=/tmp
for rep in 1 2; do
for v in base ${VARIANTS}; do
  if [ $v = base ]; then unset RS_LIB; else export RS_LIB=recommender_amd/_lib/variants/$v.so; fi
  timeout -k 10 200 python benchmarks/bench_kernels.py --only ${ONLY:-dlrm_path} > gpurun_out/abv_$v.jsonl 2> gpurun_out/abv_$v.err || { tail -20 gpurun_out/abv_$v.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/abv_$v.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$v'.ljust(10), f\"{d['avg_us']:8.1f}\", d['kernel'][:60])"
done
done
