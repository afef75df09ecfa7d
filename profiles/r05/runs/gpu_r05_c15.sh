# dependent-load latency by working-set size (tools/probe/latency_probe)
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_latency
mkdir -p $O
timeout -k 10 300 $R/tools/probe/latency_probe > $O/latency.jsonl 2> $O/latency.log || { tail -20 $O/latency.log; exit 1; }
cat $O/latency.jsonl
