# SQ counters of the DIEN kernels in the cfg3 step (run under gpurun)
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex "aux_|gru_|augru_|att_" -d gpurun_out/pmc_dien -o run --output-format csv -- python benchmarks/bench_models.py --model dien --steps 3 --warmup 1 > gpurun_out/pmc_dien.log 2>&1 || { tail -5 gpurun_out/pmc_dien.log; exit 1; }
python - <<'PY'
import csv,glob,collections
f=glob.glob('gpurun_out/pmc_dien/**/*counter_collection.csv',recursive=True)[0]
agg=collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    agg[(r['Kernel_Name'].split('(')[0][-40:],r['Counter_Name'])].append(float(r['Counter_Value']))
for k,v in sorted(agg.items()): print(k, round(sum(v)/len(v)), len(v))
PY
