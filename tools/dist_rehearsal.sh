# world-2 rehearsal of bench.py's multi-GPU path on ONE GPU (run under gpurun): two ranks share
# the card, the exchange staged through host memory (gloo) — checks that --gpus 2 takes the fused
# sharded step end to end (the driver's 8-GPU scaling run uses RCCL instead)
export TMPDIR=/tmp
RS_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps ${STEPS:-6} --warmup 2 \
  --rows ${ROWS:-40000000} --pmc 0 --compare-layerwise 0 > gpurun_out/dist_rehearsal.log 2>&1 \
  || { echo "rehearsal failed"; tail -30 gpurun_out/dist_rehearsal.log; exit 1; }
grep '"metric"' gpurun_out/dist_rehearsal.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','n_gpus','ms_per_step','scaling')}, d['config']['per_gpu_batch'], d.get('weak_scaling'), d['config']['parallelism'])"
