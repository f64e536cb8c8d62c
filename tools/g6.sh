export TMPDIR=/tmp
for gr in 2 0; do
timeout -k 10 300 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 --graph $gr > gpurun_out/bench_g$gr.log 2>&1 || { tail -20 gpurun_out/bench_g$gr.log; exit 1; }
echo graph=$gr; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_g$gr.log
done
