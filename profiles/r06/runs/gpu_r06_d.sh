# r06: trace_kernel's drain climbs from its best hit so far: the GPU suite, then a
# library A/B against the previous build (r06a), 29k and C5
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r06_d
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
L=chroma-lite_amd/chroma/_lib
bash tools/gpu_ab_libs.sh r06_ab_drain 2 "--steps 20 --warmup 5" r06a=$L/ab/libchroma_amd_r06a.so drain=$L/libchroma_amd.so || exit 1
bash tools/gpu_ab_libs.sh r06_ab_drain_c5 1 "--steps 20 --warmup 5 --detector scint" r06a=$L/ab/libchroma_amd_r06a.so drain=$L/libchroma_amd.so || exit 1
