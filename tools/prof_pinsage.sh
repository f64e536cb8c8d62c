# rocprof kernel stats of the PinSage step (run under gpurun): MODE=graph|static|dynamic
export TMPDIR=/tmp
M=${MODE:-graph}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pin_$M -o run --output-format csv -- python benchmarks/bench_models.py --model pinsage --pinsage-mode $M --steps 20 --warmup 5 > gpurun_out/prof_pin_$M.log 2>&1 || { tail -20 gpurun_out/prof_pin_$M.log; exit 1; }
python - <<PY
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_pin_$M/run_kernel_stats.csv')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print('total kernel ms', tot/1e6, 'calls', sum(int(r['Calls']) for r in rows))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:25]:
    print(f"{float(r['TotalDurationNs'])/1e3:10.1f} us {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.2f} {r['Name'][:110]}")
PY
