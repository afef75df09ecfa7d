# r06: the climb in the tail's grouped walks too (walk_segment<0, UP>): the GPU suite,
# then A/Bs -- CHR_WALK_UP 1 (lone + grouped) / 2 (lone only) / 0 (none), and the
# physics LDS copy dynamic (HEAD) vs static at the caps (staticlds), 29k
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r06_c
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
AB_ROUNDS=2 bash tools/gpu_ab_env.sh r06_ab_walkup2 "" - up= uplone=CHR_WALK_UP:2 uppair=CHR_WALK_UP:3 noup=CHR_WALK_UP:0 || exit 1
L=chroma-lite_amd/chroma/_lib
bash tools/gpu_ab_libs.sh r06_ab_lds 2 "--steps 20 --warmup 5" dyn=$L/libchroma_amd.so static=$L/ab/libchroma_amd_staticlds.so || exit 1
