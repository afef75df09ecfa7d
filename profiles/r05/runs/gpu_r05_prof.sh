#!/bin/bash
# r05 final records (run on the GPU box; GIT_HEAD in the environment):
#  1. rocprof kernel trace + stats and the HBM / L2 PMC passes of the driver's bench (29k)
#  2. bench lines of C2 / C3 / C5 and a kernel trace of C2
# usage: tools/gpu_r05_prof.sh TAG [prof|configs|both]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1; WHAT=${2:-both}
cd "$R"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
if [ "$WHAT" != configs ]; then
  bash tools/rocprof_bench.sh "gpurun_out/$T/prof29k" --steps 20 --warmup 5 || exit $?
  python3 tools/rocprof_breakdown.py "gpurun_out/$T/prof29k/trace/run_kernel_trace.csv" > "gpurun_out/$T/prof29k/breakdown.json" || exit 1
  tail -c 400 "gpurun_out/$T/prof29k/pmc_traffic.json"
fi
if [ "$WHAT" != prof ]; then
  bash tools/bench_configs.sh "gpurun_out/$T/configs" || exit $?
  for f in gpurun_out/$T/configs/*.json; do cut -c1-140 "$f"; done
  O=$R/gpurun_out/$T/prof_c2
  mkdir -p "$O"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
      python3 "$R/bench.py" --detector tiny --photons 1000000 --steps 20 --warmup 5 --no-cpu-baseline --no-count \
      > "$O/bench_trace.json" 2> "$O/bench_trace.log" || exit 1
  python3 "$R/tools/rocprof_breakdown.py" "$O/trace/run_kernel_trace.csv" > "$O/breakdown.json" || exit 1
  head -c 600 "$O/breakdown.json"
fi
