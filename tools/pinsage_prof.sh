# PinSage (cfg5) per-kernel evidence (run under gpurun): the graph step's kernel stats, then one
# FETCH_SIZE and one WRITE_SIZE PMC pass (separate runs), joined by tools/pinsage_roofline.py
export TMPDIR=/tmp
R="neighbors_kernel|agg_fwd_kernel|agg_bwd_kernel|block_emit_kernel|first_mark_kernel|first_emit_kernel|walk_kernel|pairs_gen_kernel|pair_margin|multihot"
A="benchmarks/bench_models.py --model pinsage --steps ${STEPS:-10} --warmup 3 --cpu-baseline 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pin_kt -o run --output-format csv -- python $A > gpurun_out/pin_kt.log 2>&1 || { echo "kernel trace failed"; tail -5 gpurun_out/pin_kt.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$R" -d gpurun_out/pin_$c -o run --output-format csv -- python $A > gpurun_out/pin_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pin_$c.log; exit 1; }
done
python tools/pinsage_roofline.py
