// host.cpp -- the host thread budget of the library's OpenMP regions
// (BVH builds, the wide-BVH build and record fill, the vertex merge).
//
// A GPU box shares its host: the affinity mask shows every core of the machine
// (256 on the pool's boxes) while the job's cgroup quota is far smaller (16),
// and with one process per GPU each rank should use its share of that quota.
// libgomp sizes a team by the affinity mask, so an uncapped build on 8 ranks
// would run 8 x 256 threads on 16 cores.  Every parallel region here takes
// num_threads(chr::host_threads()): chr_set_host_threads, else the usable
// cores (affinity mask capped by the cgroup v2 quota) divided by the ranks
// on this node ($LOCAL_WORLD_SIZE, set by torchrun and by bench.py).
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>

#include "../../include/chroma_amd.h"
#include "common.h"

namespace chr {
namespace {

std::atomic<int> g_threads{0};

int usable_cpus() {
    int n = 1;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::max(1, CPU_COUNT(&set));
    if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char quota[32] = {0};
        long long period = 0;
        if (std::fscanf(f, "%31s %lld", quota, &period) == 2 && period > 0 && quota[0] != 'm') {
            const long long q = std::atoll(quota);
            if (q > 0) n = std::min<long long>(n, std::max<long long>(1, q / period));
        }
        std::fclose(f);
    }
    return n;
}

int default_threads() {
    int n = usable_cpus();
    if (const char *e = std::getenv("LOCAL_WORLD_SIZE")) {
        const int w = std::atoi(e);
        if (w > 1) n = std::max(1, n / w);
    }
    return n;
}

}  // namespace

int host_threads() {
    int n = g_threads.load(std::memory_order_relaxed);
    if (n <= 0) {
        n = default_threads();
        g_threads.store(n, std::memory_order_relaxed);
    }
    return n;
}

}  // namespace chr

extern "C" int chr_set_host_threads(int32_t n) {
    if (n < 0) return chr::fail(CHR_ERR_INVALID, "chr_set_host_threads: negative count");
    chr::g_threads.store(n == 0 ? chr::default_threads() : n, std::memory_order_relaxed);
    return CHR_OK;
}

extern "C" int32_t chr_get_host_threads(void) { return chr::host_threads(); }
