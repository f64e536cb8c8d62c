# north-star step with host-side HIP runtime API trace + kernel trace (no counters): when the host
# issued each launch / stream wait vs when the GPU ran it (run under gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/ns_ht -o run --output-format csv -- python bench.py --pmc 0 --keras-line 0 --weak-secondary 0 --compare-layerwise 0 --cpu-baseline-steps 0 --steps 30 --warmup 5 > gpurun_out/ns_ht.log 2>&1 || { tail -20 gpurun_out/ns_ht.log; exit 1; }
ls gpurun_out/ns_ht/*
