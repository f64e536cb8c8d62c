# A/B of bench.py under environment switches (run under gpurun):
#   CASES="name:VAR=1,VAR2=0;name2:..." bash tools/ab_env.sh
export TMPDIR=/tmp
IFS=';' read -ra C <<< "${CASES:?}"
for c in "${C[@]}"; do
  n=${c%%:*}; vars=${c#*:}
  ( IFS=','; for kv in $vars; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 300 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 --steps ${STEPS:-40} > gpurun_out/abe_$n.json 2> gpurun_out/abe_$n.err ) || { tail -5 gpurun_out/abe_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/abe_$n.json').read().strip().splitlines()[-1]);print('$n',d['ms_per_step'])"
done
