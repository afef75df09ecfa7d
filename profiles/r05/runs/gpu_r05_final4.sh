# r05 final records at HEAD (trace kernel split into ray-record and gather instantiations): smoke, GPU suite, rocprof + PMC of the 29k bench, the bench line
set -u
R=${GRAFT_REPO_ROOT}
cd $R
WITH_PROF=1 bash tools/gpu_final.sh r05_final4 || exit 1
python3 tools/rocprof_breakdown.py gpurun_out/r05_final4/prof/trace/run_kernel_trace.csv > gpurun_out/r05_final4/prof/breakdown.json || exit 1
head -c 700 gpurun_out/r05_final4/prof/breakdown.json
