#!/bin/bash
# r04: rocprof kernel trace + stats and the HBM / L2 PMC passes of the driver's bench
# command (29k detector), then the same PMC passes for C5 (scintillator detector)
# usage: tools/gpu_r04_prof.sh TAG   (GIT_HEAD in the environment)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1
cd "$R"
bash tools/rocprof_bench.sh "gpurun_out/$T/prof29k" --steps 20 --warmup 5 || exit $?
tail -c 600 "gpurun_out/$T/prof29k/pmc_traffic.json"
