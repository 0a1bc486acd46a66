#!/bin/bash
# split diagonal step: factorisation tests, tile traces with and without the split, bench A/B
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_configs.py tests/test_gpu_dist.py -x -q \
  --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
R=$?
tail -5 $O/gputest.log
[ $R -eq 0 ] || exit $R
for n in 4096 16384; do
  timeout -k 10 120 python scripts/pt_trace.py $n > $O/pt$n.json 2>&1 || exit 1
  GPRX_PT_SPLIT=0 timeout -k 10 120 python scripts/pt_trace.py $n > $O/pt${n}_nosplit.json 2>&1 || exit 1
done
Q="--lml 0 --variance-q 0 --predict-q 0 --build-iters 0 --cpu-n 0"
timeout -k 10 300 python -u bench.py $Q > $O/bench.json 2> $O/bench.err || exit 1
GPRX_PT_SPLIT=0 timeout -k 10 300 python -u bench.py $Q > $O/bench_nosplit.json 2> $O/bench_nosplit.err || exit 1
python - <<'PY'
import json
O = "gpurun_out/r03d"
for f in ("pt4096", "pt4096_nosplit", "pt16384", "pt16384_nosplit"):
    d = json.load(open(f"{O}/{f}.json"))
    print(f, d["ms_devbench"], d["span_us"], d.get("chain_period_us"), d["DIAGX"]["exec_us_mean"],
          {k: round(v["exec_us_mean"], 1) for k, v in d.items() if k.startswith("TPART_c")})
for f in ("bench", "bench_nosplit"):
    d = json.load(open(f"{O}/{f}.json"))
    print(f, round(d["value"], 2), round(d["roofline"]["avg_launch_us"], 1),
          {k: round(v.get("value") or 0, 2) for k, v in (d.get("configs") or {}).items()})
PY
