# round-4 timelines (run under gpurun): one north-star step and one DIEN step as kernel
# sequences (tools/step_trace.py), then the PinSage roofline passes and the cfg3/cfg4 profiles
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ns_kt -o run --output-format csv -- python bench.py --pmc 0 --keras-line 0 --weak-secondary 0 --compare-layerwise 0 --cpu-baseline-steps 0 --steps 30 --warmup 5 > gpurun_out/ns_kt.log 2>&1 || { tail -20 gpurun_out/ns_kt.log; exit 1; }
f=$(find gpurun_out/ns_kt -name "*kernel_trace.csv" | head -1)
python tools/step_trace.py "$f" --marker dlrm_train_chunk > gpurun_out/ns_step_trace.txt && head -60 gpurun_out/ns_step_trace.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/dien_kt -o run --output-format csv -- python benchmarks/bench_models.py --model dien --dien-mode eager --steps 4 --warmup 2 > gpurun_out/dien_kt.log 2>&1 || { tail -20 gpurun_out/dien_kt.log; exit 1; }
f=$(find gpurun_out/dien_kt -name "*kernel_trace.csv" | head -1)
python tools/step_trace.py "$f" --marker gru_fwd_kernel > gpurun_out/dien_step_trace.txt && tail -3 gpurun_out/dien_step_trace.txt
bash tools/r04_pinsage_prof.sh || exit 1
bash tools/r04_models_prof.sh
