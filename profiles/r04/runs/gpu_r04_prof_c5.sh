#!/bin/bash
# r04: rocprof kernel stats + HBM / L2 PMC passes of the C5 bench (scintillator detector,
# 10 M photons), usage: tools/gpu_r04_prof_c5.sh TAG (GIT_HEAD in the environment)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
bash tools/rocprof_bench.sh "gpurun_out/$1/prof_c5" --detector scint --photons 10000000 --steps 10 --warmup 3 || exit $?
tail -c 400 "gpurun_out/$1/prof_c5/pmc_traffic.json"
