export TMPDIR=/tmp
for g in 0 1 2; do
timeout -k 10 300 python bench.py --graph $g --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 --steps 40 > gpurun_out/bg$g.json 2> gpurun_out/bg$g.err || { tail -5 gpurun_out/bg$g.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bg$g.json').read().strip().splitlines()[-1]);print($g, d['ms_per_step'], d['value'])"
done
