export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/bench_models.py --model dien > gpurun_out/d0.jsonl 2>/dev/null || exit 1
cut -c1-120 gpurun_out/d0.jsonl
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune_dien%d.csv timeout -k 10 600 python benchmarks/bench_models.py --model dien > gpurun_out/d1.jsonl 2>/dev/null || exit 1
cut -c1-120 gpurun_out/d1.jsonl
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune_dien%d.csv timeout -k 10 300 python benchmarks/bench_models.py --model dien > gpurun_out/d2.jsonl 2>/dev/null || exit 1
cut -c1-120 gpurun_out/d2.jsonl
