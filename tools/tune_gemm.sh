export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline-steps 0 --pmc 0 > gpurun_out/t0.log 2>&1 || { tail -5 gpurun_out/t0.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/t0.log
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 500 python bench.py --steps 20 --warmup 5 --cpu-baseline-steps 0 --pmc 0 > gpurun_out/t1.log 2>&1 || { tail -20 gpurun_out/t1.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/t1.log
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline-steps 0 --pmc 0 > gpurun_out/t2.log 2>&1 || { tail -20 gpurun_out/t2.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/t2.log
ls -la gpurun_out/
