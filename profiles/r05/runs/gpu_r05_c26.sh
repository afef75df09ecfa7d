# trace_kernel LDS split between stack top (SL) and parked-leaf queue (LEAFQ): library A/B
set -u
R=${GRAFT_REPO_ROOT}
cd $R
L=chroma-lite_amd/chroma/_lib/ab
bash tools/gpu_ab_libs.sh r05_ab_SL 2 "--steps 20 --warmup 5" s12_16=$L/s12_16.so s14_12=$L/s14_12.so s10_20=$L/s10_20.so s16_8=$L/s16_8.so || exit 1
