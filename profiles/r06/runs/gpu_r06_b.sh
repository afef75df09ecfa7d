# r06: the reference nearest-hit rule + culling margin (ref_beats / ref_cut) and the
# dynamic physics LDS: smoke, the GPU suite, then the driver's bench command cold
# with the round-5 parity sample (9,897,030 photons)
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r06_b
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
timeout -k 10 600 python3 "$R/bench.py" --steps 20 --warmup 5 --parity-photons 9897030 > "$O/bench.json" 2> "$O/bench.log" || { tail -5 "$O/bench.log"; exit 1; }
cut -c1-300 "$O/bench.json"
