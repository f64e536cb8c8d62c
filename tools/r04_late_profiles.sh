# round 4: kernel profiles of the DIEN and ESMM steps on the final tree (gpurun)
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
for m in dien esmm; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_${m}_late -o run -- python $GRAFT_REPO_ROOT/benchmarks/bench_models.py --model $m --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_${m}_late.log 2>&1 || { echo "$m prof failed"; exit 1; }
  echo "$m prof ok"
done
