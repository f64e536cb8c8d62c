# SQ counters of the DIEN kernels in the cfg3 step (run under gpurun); summary by
# tools/pmc_summary.py. The run must exit 0 (round 6: KernelTimer records no events inside a
# graph capture, which is what made bench_models exit non-zero under --pmc before).
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_dien
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex "aux_|gru_|augru_|att_" -d gpurun_out/pmc_dien -o run --output-format csv -- python benchmarks/bench_models.py --model dien --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/pmc_dien.log 2>&1 || { echo "rocprofv3 run failed"; tail -5 gpurun_out/pmc_dien.log; exit 1; }
set -- gpurun_out/pmc_dien/*counter_collection.csv
f=$1
[ -f "$f" ] || { echo "no counter file"; tail -5 gpurun_out/pmc_dien.log; exit 1; }
python tools/pmc_summary.py "$f"
