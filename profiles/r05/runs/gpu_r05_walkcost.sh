# per-step walk-cost histograms (counting trace variant, host-driven steps) of the 29k bench
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_walkcost
mkdir -p $O
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
CHR_TRACE_STEPS=1 CHR_PROPAGATE_VARIANT=5 timeout -k 10 600 python3 -u $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline \
  --no-count --sequential-steps 0 --timing-steps 0 --no-pipeline > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
grep -A2 "chr_propagate: step" $O/bench.log | head -80
