# A/B of the north-star step's stream schedule (run under gpurun): each variant is one bench.py
# run without the PMC / secondary lines; prints ms/step (median, p10) and the in-step spans.
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, env..., -- bench args
  name=$1; shift
  envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --pmc 0 --keras-line 0 --weak-secondary 0 \
    --compare-layerwise 0 --cpu-baseline-steps 0 --steps 200 "$@" > gpurun_out/stepab_$name.json 2> gpurun_out/stepab_$name.err || { echo "$name failed"; tail -5 gpurun_out/stepab_$name.err; return 1; }
  python - "$name" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/stepab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
k = d.get("kernels") or {}
dist = d.get("step_ms_distribution") or {}
print(f"{sys.argv[1]:14s} ms/step {d['ms_per_step']:.4f} median {dist.get('median')} "
      f"p10 {dist.get('p10')} | " +
      " ".join(f"{n.replace('rs_', '')[:18]} {v['avg_us']}" for n, v in k.items()))
PY
}
for rep in ${REPS:-1 2}; do
  for v in ${VARIANTS:-base graph2}; do
    case $v in
      base) run base X=1 -- || exit 1 ;;
      graph2) run graph2 X=1 -- --graph 2 || exit 1 ;;
      prefetch) run prefetch X=1 -- --prefetch 1 || exit 1 ;;
      waitsort) run waitsort RS_TRAIN_WAITS_SORT=1 -- || exit 1 ;;
      mainprio) run mainprio X=1 -- --prio 1 || exit 1 ;;
      sysev) run sysev RS_DEVICE_EVENTS=0 -- || exit 1 ;;
    esac
  done
done
