# SQ / instruction-mix counters of the fused train kernel (KREGEX, default dlrm_train_chunk), two passes (run
# under gpurun); each pass within the per-block counter limits
export TMPDIR=/tmp
run() {
  timeout -s KILL 90 rocprofv3 --pmc $2 --kernel-include-regex ${KREGEX:-dlrm_train_chunk} -d gpurun_out/pmc_$1 -o run --output-format csv -- python benchmarks/bench_kernels.py --only dlrm_path --iters 2 > gpurun_out/pmc_$1.log 2>&1 || { tail -5 gpurun_out/pmc_$1.log; exit 1; }
}
run a "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES" && \
run b "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD" && \
python - <<'PY'
import csv,glob,collections
for p in ("a","b"):
    f=glob.glob(f'gpurun_out/pmc_{p}/**/*counter_collection.csv',recursive=True)[0]
    agg=collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for k,v in sorted(agg.items()): print(f"{k:28s} {sum(v)/len(v):16,.0f}  (mean of {len(v)} launches)")
PY
