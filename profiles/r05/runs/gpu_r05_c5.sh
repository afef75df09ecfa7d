set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_c5
mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
if ! timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; then
  tail -30 $O/pytest_gpu.log
  grep -q "^FAILED tests/test_gpu_batches.py::test_switches" $O/pytest_gpu.log && \
    timeout -k 10 600 python -u tools/diag_switch.py base= v5=CHR_PROPAGATE_VARIANT:5 wo0=CHR_WALK_ORDER:0 > $O/diag.jsonl 2> $O/diag.log
  cat $O/diag.jsonl
  exit 1
fi
tail -1 $O/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u $R/bench.py --detector scint --photons 10000000 --steps 10 --warmup 3 > $O/bench_scint.json 2> $O/bench_scint.log || { tail -20 $O/bench_scint.log; exit 1; }
cut -c1-300 $O/bench_scint.json
