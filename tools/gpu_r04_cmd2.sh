set -u
T="tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_batches.py"
CHR_TRACE_LAYOUT=3 timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04t3_lay3.log 2>&1 || { tail -30 gpurun_out/r04t3_lay3.log; exit 1; }
tail -1 gpurun_out/r04t3_lay3.log
CHR_TRACE_LAYOUT=4 timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04t3_lay4.log 2>&1 || { tail -30 gpurun_out/r04t3_lay4.log; exit 1; }
tail -1 gpurun_out/r04t3_lay4.log
bash tools/gpu_ab_env.sh r04ab3 "" - base= lay3=CHR_TRACE_LAYOUT:3 lay4=CHR_TRACE_LAYOUT:4 || exit 1
bash tools/gpu_ab_libs.sh r04libs2 2 "--steps 20 --warmup 5" walk1=chroma-lite_amd/chroma/_lib/ab/libchroma_amd_walk1.so walk2=chroma-lite_amd/chroma/_lib/ab/libchroma_amd_walk2.so
