export TMPDIR=/tmp
for m in ${MODES:-0 128 176 192 240}; do
RS_DX_DEBUG=$m timeout -k 10 120 python benchmarks/bench_kernels.py --only dlrm_path 2>/dev/null | head -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print($m, d['avg_us'])" || exit 1
done
