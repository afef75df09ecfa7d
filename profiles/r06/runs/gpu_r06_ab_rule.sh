# r06 library A/B: r05 kernels (base) vs the reference nearest-hit rule with the
# culling margin (new, HEAD) vs the rule without the margin (nomargin), 29k then C5
set -u
R=${GRAFT_REPO_ROOT}
cd $R
L=chroma-lite_amd/chroma/_lib
bash tools/gpu_ab_libs.sh r06_ab_rule 2 "--steps 20 --warmup 5" base=$L/ab/libchroma_amd_base.so new=$L/libchroma_amd.so nomargin=$L/ab/libchroma_amd_nomargin.so || exit 1
bash tools/gpu_ab_libs.sh r06_ab_rule_c5 1 "--steps 20 --warmup 5 --detector scint" base=$L/ab/libchroma_amd_base.so new=$L/libchroma_amd.so || exit 1
