# flat machinery removed + early binning of the next batch (CHR_EARLY_BIN_SLOT): GPU suite, A/Bs
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_c9
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/gpu_ab_libs.sh r05_ab_clean 1 "--steps 20 --warmup 5" flat=chroma-lite_amd/chroma/_lib/ab/flat.so clean=chroma-lite_amd/chroma/_lib/ab/clean.so || exit 1
AB_ROUNDS=2 bash tools/gpu_ab_env.sh r05_ab_early "" - e0=CHR_EARLY_BIN_SLOT:0 e3=CHR_EARLY_BIN_SLOT:3 e5=CHR_EARLY_BIN_SLOT:5 e7=CHR_EARLY_BIN_SLOT:7 || exit 1
