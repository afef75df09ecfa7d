# device region profiles: C5 (scintillator) and 29k
set -u
R=${GRAFT_REPO_ROOT}
cd $R
bash tools/gpu_devprof.sh r05_dp_c5 --detector scint --photons 10000000 || exit 1
bash tools/gpu_devprof.sh r05_dp_29k || exit 1
