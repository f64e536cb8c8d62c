# DeepFM graph-captured Keras-Adam step: parity + cfg1 bench both modes (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_deepfm_gpu.py -q -x --timeout 400 --timeout-method thread > gpurun_out/deepfm_t.log 2>&1 || { tail -30 gpurun_out/deepfm_t.log; exit 1; }
tail -1 gpurun_out/deepfm_t.log
for mode in graph eager graph; do timeout -k 10 300 python benchmarks/bench_models.py --model deepfm --deepfm-mode $mode --steps 50 --warmup 5 2>/dev/null | tail -1 | cut -c1-200; done
