# world-2 rehearsal of bench.py's multi-GPU path on ONE GPU (run under gpurun): two ranks,
# gloo transport staged through host memory (RCCL needs one GPU per rank)
export TMPDIR=/tmp RS_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps ${STEPS:-5} --warmup 2 --pmc 0 --cpu-baseline-steps 0 --compare-layerwise 0 ${BENCH_ARGS:-} > gpurun_out/w2.log 2>&1 || { tail -30 gpurun_out/w2.log; exit 1; }
tail -1 gpurun_out/w2.log | cut -c1-600
