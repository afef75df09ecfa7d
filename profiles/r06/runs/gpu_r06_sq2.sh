# r06: the second SQ-counter pass VERDICT r05 item 3 names (LDS instructions, LDS issue and
# stall cycles, bank conflicts, VALU thread cycles, scalar-memory instructions) on the
# final kernels (44368146), the bench workload, per dispatch class (tools/sq_summary.py)
set -u
R=${GRAFT_REPO_ROOT}
cd "$R"
SQ_WANT="SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM" \
    bash tools/gpu_sq_pmc.sh r06_sq2 || exit 1
python3 tools/sq_summary.py gpurun_out/r06_sq2/sq/run_counter_collection.csv > gpurun_out/r06_sq2/sq_summary.json || exit 1
cat gpurun_out/r06_sq2/sq_summary.json
