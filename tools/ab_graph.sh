# A/B of bench modes (run under gpurun): MODES="name:args;name:args"
export TMPDIR=/tmp
IFS=';' read -ra M <<< "${MODES:-eager:--graph 0;graph1:--graph 1;graph2:--graph 2}"
for m in "${M[@]}"; do
n=${m%%:*}; a=${m#*:}
timeout -k 10 300 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 --steps 40 $a > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -20 gpurun_out/ab_$n.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/ab_$n.json').read().strip().splitlines()[-1]);print('$n ms/step',d['ms_per_step'])"
done
