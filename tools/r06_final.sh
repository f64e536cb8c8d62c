# Round-6 final records (run under gpurun): the default bench line (100 steps), the driver's
# short form (20 steps after 5), and the kernel stats of the bench under rocprofv3
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --steps 100 --warmup 10 > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err || { tail -5 gpurun_out/fin_bench.err; exit 1; }
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/fin_bench20.json 2> gpurun_out/fin_bench20.err || { tail -5 gpurun_out/fin_bench20.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 --pmc 0 --compare-layerwise 0 --keras-line 0 --weak-secondary 0 > gpurun_out/fin_prof.log 2>&1 || { tail -5 gpurun_out/fin_prof.log; exit 1; }
