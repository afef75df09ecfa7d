# pipelined ray refills as the only ray-record path: GPU parity + batch tests, then library A/B against the previous build
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_c22
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_batches.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab_libs.sh r05_ab_pipe_libs 3 "--steps 20 --warmup 5" base=chroma-lite_amd/chroma/_lib/ab/base.so pipe=chroma-lite_amd/chroma/_lib/ab/pipe.so || exit 1
bash tools/gpu_ab_libs.sh r05_ab_pipe_libs_c5 2 "--steps 20 --warmup 5 --detector scint" base=chroma-lite_amd/chroma/_lib/ab/base.so pipe=chroma-lite_amd/chroma/_lib/ab/pipe.so || exit 1
