# trace_kernel triangle-step threshold F (4..7 of 8 walking lanes with parked leaves): library A/B, 29k + scintillator
set -u
R=${GRAFT_REPO_ROOT}
cd $R
L=chroma-lite_amd/chroma/_lib/ab
bash tools/gpu_ab_libs.sh r05_ab_F 2 "--steps 20 --warmup 5" f6=$L/f6.so f4=$L/f4.so f5=$L/f5.so f7=$L/f7.so || exit 1
bash tools/gpu_ab_libs.sh r05_ab_F_c5 1 "--steps 20 --warmup 5 --detector scint" f6=$L/f6.so f5=$L/f5.so f7=$L/f7.so || exit 1
