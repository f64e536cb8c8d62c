# SQ counters of the fused forward kernel (run under gpurun)
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --kernel-include-regex "${KREGEX:-dlrm_fwd_dx_pipe}" -d gpurun_out/pmc_dx -o run --output-format csv -- python benchmarks/bench_kernels.py --only dlrm_path --iters 2 > gpurun_out/pmc_dx.log 2>&1 || { tail -5 gpurun_out/pmc_dx.log; exit 1; }
python - <<'PY'
import csv,glob,collections
f=glob.glob('gpurun_out/pmc_dx/**/*counter_collection.csv',recursive=True)[0]
agg=collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    agg[(r['Kernel_Name'][:60],r['Counter_Name'])].append(float(r['Counter_Value']))
for k,v in sorted(agg.items()): print(k, sum(v)/len(v), len(v))
PY
