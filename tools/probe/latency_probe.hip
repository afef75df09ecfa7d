// Dev tool: dependent-load latency of one wave on MI355X (pointer chase), by
// working-set size -- L1 (TCP), L2, MALL, HBM -- for 16-byte vector loads
// (global_load_dwordx4, as the walk's node loads) and the same chase with the
// whole wave's 64 lanes loading 64 different lines per step.
// Build: hipcc --offload-arch=gfx950 -O3 -o latency_probe latency_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include <algorithm>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void chase(const u32x4 *a, unsigned steps, unsigned lines, unsigned long long *out, unsigned *sink,
                      int spread) {
    unsigned p = spread ? ((threadIdx.x * 7919u) % lines) * 8u : 0u;
    unsigned acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (unsigned i = 0; i < steps; ++i) {
        const u32x4 v = *(const __attribute__((address_space(1))) u32x4 *)(a + p);
        p = v.x;
        acc += v.y;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[0] = t1 - t0;
    sink[threadIdx.x] = acc + p;
}

int main() {
    const size_t sizes_kb[] = {8, 24, 256, 2048, 3072, 16384, 65536, 262144, 2097152};
    unsigned long long *d_out;
    unsigned *d_sink;
    hipMalloc(&d_out, 8);
    hipMalloc(&d_sink, 256 * 4);
    for (int spread = 0; spread < 2; ++spread)
        for (size_t kb : sizes_kb) {
            const size_t n = kb * 1024 / 16;   // 16-byte elements
            // a random cycle over elements spaced one 128-byte line apart
            const size_t lines = std::max<size_t>(2, n / 8);
            std::vector<unsigned> perm(lines);
            for (size_t i = 0; i < lines; ++i) perm[i] = (unsigned)i;
            std::mt19937 rng(1);
            std::shuffle(perm.begin() + 1, perm.end(), rng);
            std::vector<u32x4> h(n);
            for (size_t i = 0; i < lines; ++i) {
                const unsigned from = perm[i] * 8, to = perm[(i + 1) % lines] * 8;
                h[from] = u32x4{to, 1u, 0u, 0u};
            }
            u32x4 *d;
            hipMalloc(&d, n * 16);
            hipMemcpy(d, h.data(), n * 16, hipMemcpyHostToDevice);
            const unsigned steps = 4096;
            unsigned long long cyc[2] = {0, 0};
            for (int rep = 0; rep < 2; ++rep) {   // rep 0 warms (caches that hold the set)
                hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d, steps, (unsigned)lines, d_out, d_sink, spread);
                hipMemcpy(&cyc[rep], d_out, 8, hipMemcpyDeviceToHost);
            }
            printf("{\"spread\": %d, \"kb\": %zu, \"cycles_per_load_cold\": %.1f, \"cycles_per_load\": %.1f}\n", spread,
                   kb, (double)cyc[0] / steps, (double)cyc[1] / steps);
            fflush(stdout);
            hipFree(d);
        }
    int khz = 0;
    hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, 0);
    printf("{\"clock_khz\": %d}\n", khz);
    return 0;
}
