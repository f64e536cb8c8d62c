# PinSage cfg5 roofline evidence (run under gpurun): kernel stats of the whole-step graph at the
# ML-20M shape, then FETCH_SIZE / WRITE_SIZE PMC passes (separate runs, as the MI355X guide says)
# over the sampling / aggregation kernels; tools/pinsage_roofline.py joins them.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pin_kt -o run --output-format csv -- python benchmarks/bench_models.py --model pinsage --pinsage-mode graph_all --steps 20 --warmup 5 > gpurun_out/pin_kt.log 2>&1 || { tail -20 gpurun_out/pin_kt.log; exit 1; }
RE="neighbors_kernel|agg_fwd_kernel|agg_bwd_kernel|block_emit_kernel|first_mark_kernel|first_emit_kernel|walk_kernel|pairs_gen_kernel"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$RE" -d gpurun_out/pin_$c -o run --output-format csv -- python benchmarks/bench_models.py --model pinsage --pinsage-mode static --steps 4 --warmup 1 > gpurun_out/pin_$c.log 2>&1 || { tail -20 gpurun_out/pin_$c.log; exit 1; }
done
python tools/pinsage_roofline.py > gpurun_out/pin_roofline.txt && cat gpurun_out/pin_roofline.txt
