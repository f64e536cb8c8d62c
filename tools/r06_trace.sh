# Round-6 kernel records (run under gpurun): the sort + apply probe under rocprofv3 --stats and a
# 30-step bench kernel trace for the step timeline (tools/step_timeline.py)
export TMPDIR=/tmp
mkdir -p gpurun_out
B="--steps 30 --warmup 5 --cpu-baseline-steps 0 --pmc 0 --compare-layerwise 0 --keras-line 0 --weak-secondary 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_sort -o run -- python3 tools/probe_sorted_grad.py > gpurun_out/${TAG}_sort.log 2>&1 || { tail -5 gpurun_out/${TAG}_sort.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_tl -o tl -- python3 bench.py $B > gpurun_out/${TAG}_tl.log 2>&1 || { tail -5 gpurun_out/${TAG}_tl.log; exit 1; }
