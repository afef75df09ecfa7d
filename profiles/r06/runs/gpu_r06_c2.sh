# r06: where C2 (demo.tiny(), 1 M photons) lost 2% against round 5: library A/B of the
# round-5 kernels (base), this round's before the climb without the culling margin
# (nomargin, not exact) and HEAD, two rounds, photons hashed
set -u
R=${GRAFT_REPO_ROOT}
cd "$R"
bash tools/gpu_ab_libs.sh r06_ab_c2 2 "--detector tiny --photons 1000000 --steps 20 --warmup 5" \
    base=chroma-lite_amd/chroma/_lib/ab/libchroma_amd_base.so \
    nomargin=chroma-lite_amd/chroma/_lib/ab/libchroma_amd_nomargin.so \
    head=chroma-lite_amd/chroma/_lib/libchroma_amd.so || exit 1
