# Bench lines of C2 / C3 / C5 from the committed tree, and a rocprofv3 kernel
# trace of C2 (why its trace roofline fraction is low).  usage: TAG (e.g. the sha)
set -u
R=${GRAFT_REPO_ROOT}
T=$1
cd $R
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
bash tools/bench_configs.sh gpurun_out/r05_configs_$T || exit 1
for f in gpurun_out/r05_configs_$T/*.json; do cut -c1-160 $f; done
O=$R/gpurun_out/r05_prof_c2_$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --detector tiny --photons 1000000 --steps 20 --warmup 5 --no-cpu-baseline --no-count \
    > $O/bench_trace.json 2> $O/bench_trace.log || exit 1
ls -R $O | head -20
