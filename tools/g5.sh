export TMPDIR=/tmp
timeout -k 10 300 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 --batch 2048 --rows 4000000 > gpurun_out/b_small.log 2>&1 || { tail -20 gpurun_out/b_small.log; exit 1; }
echo small; grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_small.log
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv timeout -k 10 500 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 > gpurun_out/t1.log 2>&1 || { tail -20 gpurun_out/t1.log; exit 1; }
echo tune; grep -o '"ms_per_step": [0-9.]*' gpurun_out/t1.log
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv timeout -k 10 200 python bench.py --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 > gpurun_out/t2.log 2>&1 || { tail -20 gpurun_out/t2.log; exit 1; }
echo tuned; grep -o '"ms_per_step": [0-9.]*' gpurun_out/t2.log
