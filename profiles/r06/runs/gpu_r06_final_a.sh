# r06 round-end records, part 1: smoke, the GPU suite, the rocprofv3 kernel trace and
# the HBM / L2 PMC passes of the driver's bench command (profiles/latest_pmc.json),
# and the SQ-counter pass of the same workload
set -u
R=${GRAFT_REPO_ROOT}
TAG=${1:-r06_final}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
bash "$R/tools/rocprof_bench.sh" "gpurun_out/$TAG/prof" --steps 20 --warmup 5 || exit $?
cp "$O/prof/pmc_traffic.json" "$R/profiles/latest_pmc.json" || exit $?
python3 "$R/tools/rocprof_breakdown.py" "$O/prof/trace/run_kernel_trace.csv" > "$O/prof/breakdown.json" || exit 1
bash "$R/tools/gpu_sq_pmc.sh" ${TAG}_sq || exit 1
