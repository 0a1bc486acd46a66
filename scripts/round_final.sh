# End-of-round measurement set on one GPU box (each step bounded; stops at the first failure):
# GPU tests, the default bench line (with the CPU baseline), the other configurations, the
# tile-engine traces at N = 4096 / 16384 and the diagonal-factor microbenchmark.
set -e
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/gputest.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/final/bench.log 2>&1
timeout -k 10 300 python scripts/bench_configs.py --steps 10 > gpurun_out/final/configs.jsonl 2>&1
timeout -k 10 300 python scripts/bench_sparse.py > gpurun_out/final/sparse.jsonl 2>&1
timeout -k 10 120 python scripts/pt_trace.py 4096 > gpurun_out/final/pt4096.json 2>&1
timeout -k 10 120 python scripts/pt_trace.py 16384 > gpurun_out/final/pt16384.json 2>&1
timeout -k 10 120 python scripts/diag_bench.py > gpurun_out/final/diag_bench.json 2>&1
echo done
