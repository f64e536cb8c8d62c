# Round-6 profile records (run under gpurun): the north-star sort alone under rocprofv3 --stats
# (tools/probe_sorted_grad.py: the slot-segmented sort and the apply on the bench's ids), the
# path's SQ counters inside bench.py steps (tools/pmc_path.sh) and the train kernel's counters
# (tools/pmc_train.sh)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sortstats -o run -- python3 tools/probe_sorted_grad.py > gpurun_out/sortstats.log 2>&1 || { tail -5 gpurun_out/sortstats.log; exit 1; }
bash tools/pmc_path.sh > gpurun_out/pmc_path_summary.txt 2>&1 || { tail -5 gpurun_out/pmc_path_summary.txt; exit 1; }
bash tools/pmc_train.sh > gpurun_out/pmc_train_summary.txt 2>&1 || { tail -5 gpurun_out/pmc_train_summary.txt; exit 1; }
