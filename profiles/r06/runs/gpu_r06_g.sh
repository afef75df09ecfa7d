# r06: is the pair walk's tester still worth its waves now that the climb walks ahead of
# it (long_paired_step_fraction 0.0 in the round-end records)?  Env A/B: pair (default)
# vs none (CHR_PAIR_WALK=0: the idle waves of a tail workgroup exit instead of polling
# the mailbox), 29k two rounds and C5 one round, photons hashed
set -u
R=${GRAFT_REPO_ROOT}
cd "$R"
AB_ROUNDS=2 bash tools/gpu_ab_env.sh r06_ab_nopair "" - pair= nopair=CHR_PAIR_WALK:0 || exit 1
AB_ROUNDS=1 AB_ARGS="--detector scint" bash tools/gpu_ab_env.sh r06_ab_nopair_c5 "" - pair= nopair=CHR_PAIR_WALK:0 || exit 1
