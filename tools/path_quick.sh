# isolated embedding-path launches only (run under gpurun)
export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/bench_kernels.py --only dlrm_path > gpurun_out/path.jsonl 2> gpurun_out/path.err || { tail -20 gpurun_out/path.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/path.jsonl'):
    d=json.loads(l); print(f\"{d['avg_us']:9.1f} us  {d['frac_of_hbm_peak']:.3f}  {d['kernel']}\")"
