# flat-walk machinery removed (no sub-walks, no cut, no rank map on the device): GPU suite + library A/B
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_c8
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/gpu_ab_libs.sh r05_ab_clean 2 "--steps 20 --warmup 5" flat=chroma-lite_amd/chroma/_lib/ab/flat.so clean=chroma-lite_amd/chroma/_lib/ab/clean.so || exit 1
