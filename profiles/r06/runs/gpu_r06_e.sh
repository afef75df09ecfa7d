# r06: the binning sort on the Hilbert index's top 16 bits (CHR_BIN_SORT_LOW=6: two
# radix passes instead of three) vs all 22, in-process A/B on 29k; then the parity
# sweep over six more photon seeds (tools/parity_sweep.py, 6 x 10 M photons)
set -u
R=${GRAFT_REPO_ROOT}
cd "$R"
AB_ROUNDS=2 bash tools/gpu_ab_env.sh r06_ab_bsort "" - b22= b16=CHR_BIN_SORT_LOW:6 || exit 1
bash profiles/r06/runs/gpu_r06_sweep.sh || exit 1
