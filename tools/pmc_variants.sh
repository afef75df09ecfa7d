#!/bin/bash
# PMC passes (one counter group per run) over an in-process A/B of kernel
# variants (tools/ab_variants.py); run on the GPU box.
# usage: tools/pmc_variants.sh OUTDIR VARIANTS [detector] [photons]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1; V=$2; DET=${3:-demo}; N=${4:-4000000}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$R/tools/ab_variants.py" --detector $DET --photons $N --variants $V --rounds 1 > "$OUT/p$i.log" 2>&1 || exit $?
done
python3 "$R/tools/pmc_summary.py" "$OUT/p1" "$OUT/p2" > "$OUT/summary.txt"
