# r06 A/Bs: libraries -- r05 kernels (base) vs HEAD (the reference nearest-hit rule
# with its culling margin, walk_up, dynamic physics LDS: new) vs HEAD without the
# margin (nomargin) -- on 29k; walk_up on / off in HEAD (env, 29k); base vs new on C5
set -u
R=${GRAFT_REPO_ROOT}
cd $R
L=chroma-lite_amd/chroma/_lib
bash tools/gpu_ab_libs.sh r06_ab_rule 2 "--steps 20 --warmup 5" base=$L/ab/libchroma_amd_base.so new=$L/libchroma_amd.so nomargin=$L/ab/libchroma_amd_nomargin.so || exit 1
AB_ROUNDS=2 bash tools/gpu_ab_env.sh r06_ab_walkup "" - up= noup=CHR_WALK_UP:0 || exit 1
bash tools/gpu_ab_libs.sh r06_ab_rule_c5 1 "--steps 20 --warmup 5 --detector scint" base=$L/ab/libchroma_amd_base.so new=$L/libchroma_amd.so || exit 1
