# split-bf16 GEMM: parity vs float64 (both stage variants), then the A/B against the library GEMMs
export TMPDIR=/tmp
mkdir -p gpurun_out
for st in 1 2; do
RS_GEMM_STAGES=$st timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/gemm_t$st.log 2>&1 || { tail -30 gpurun_out/gemm_t$st.log; exit 1; }
tail -1 gpurun_out/gemm_t$st.log
RS_GEMM_STAGES=$st timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench$st.jsonl 2> gpurun_out/gemm_bench$st.err || { tail -20 gpurun_out/gemm_bench$st.err; exit 1; }
cut -c1-200 gpurun_out/gemm_bench$st.jsonl
done
