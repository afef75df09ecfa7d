# hit record (trace publishes code + e1 x e3; shade gathers no triangle record): GPU suite + library A/B
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_c6
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/gpu_ab_libs.sh r05_ab_hitx 2 "--steps 20 --warmup 5" base=chroma-lite_amd/chroma/_lib/ab/base.so hitx=chroma-lite_amd/chroma/_lib/ab/hitx.so || exit 1
bash tools/gpu_ab_libs.sh r05_ab_hitx_c5 1 "--steps 20 --warmup 5 --detector scint" base=chroma-lite_amd/chroma/_lib/ab/base.so hitx=chroma-lite_amd/chroma/_lib/ab/hitx.so || exit 1
