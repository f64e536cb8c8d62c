# SQ counters of the north-star path's kernels inside bench.py steps (run under gpurun): the
# train kernel, the slot-segmented sort, the apply walk (+ its fix-up); one pass, summary by
# tools/pmc_summary.py (VGPRs / LDS per workgroup, MFMA busy, wait shares, VALU per wave)
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_path
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex "dlrm_train_chunk|slot_sort_|radix_|seg_group|seg_fixup" -d gpurun_out/pmc_path -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 --keras-line 0 > gpurun_out/pmc_path.log 2>&1
set -- gpurun_out/pmc_path/*counter_collection.csv
f=$1
[ -f "$f" ] || { echo "no counter file"; tail -5 gpurun_out/pmc_path.log; exit 1; }
python tools/pmc_summary.py "$f"
