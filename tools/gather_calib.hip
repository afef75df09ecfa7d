// gather_calib.hip -- calibrate rocprofv3 FETCH_SIZE on gfx950 for the access
// shapes of the BVH walk (VERDICT r01 "what's weak" 3: the x2 FETCH correction
// of MI355X_MICROARCH.md is stated for wide coalesced streams only).
//
// Each kernel reads a KNOWN set of bytes from an 8 GiB buffer (far past the
// 256 MiB Infinity Cache, cold: every kernel touches its own region):
//   stream16      coalesced 16 B/lane stream (the guide's calibration case)
//   gather<R,S>   one lane per record: R bytes (R/16 uint4 loads) of record
//                 idx at stride S, idx a permutation (each record once)
//   gather_bc<8>  8 lanes load the same 96-byte record (the group walk's
//                 broadcast node fetch)
// and the host prints, per kernel, the bytes requested and the 64-B sectors /
// 128-B lines they span.  FETCH_SIZE (KiB) of the same dispatches is read from
// rocprofv3's counter CSV by tools/gather_calib.py.
//
// build: hipcc --offload-arch=gfx950 -O3 -o gather_calib tools/gather_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

constexpr int BLOCK = 256;

__global__ __launch_bounds__(BLOCK) void stream16(const uint4 *src, size_t n, uint32_t *sink) {
    const size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    uint32_t acc = 0;
    for (size_t k = i; k < n; k += (size_t)gridDim.x * BLOCK) {
        const uint4 v = src[k];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[i] = acc;   // practically never: no write traffic
}

// record index of work-item i: a permutation of [0, nrec) (P odd, nrec a power of two)
__device__ __host__ inline uint64_t perm(uint64_t i, uint64_t nrec) { return (i * 2654435761ull + 12345ull) & (nrec - 1); }

template <int R, int S>
__global__ __launch_bounds__(BLOCK) void gather(const char *base, uint64_t nrec, uint32_t n, uint32_t *sink) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint4 *p = (const uint4 *)(base + perm(i, nrec) * S);
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < R / 16; ++k) {
        const uint4 v = p[k];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[i] = acc;
}

template <int G>
__global__ __launch_bounds__(BLOCK) void gather_bc(const char *base, uint64_t nrec, uint32_t n, uint32_t *sink) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i / G >= n) return;
    const uint4 *p = (const uint4 *)(base + perm(i / G, nrec) * 96);
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const uint4 v = p[k];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[i] = acc;
}

struct Spans { uint64_t bytes, sectors64, lines128; };

static Spans spans(uint64_t off0, uint64_t nrec, uint32_t n, int R, int S) {
    std::set<uint64_t> s64, l128;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t a = off0 + perm(i, nrec) * (uint64_t)S;
        for (uint64_t b = a / 64; b <= (a + R - 1) / 64; ++b) s64.insert(b);
        for (uint64_t b = a / 128; b <= (a + R - 1) / 128; ++b) l128.insert(b);
    }
    return Spans{(uint64_t)n * R, (uint64_t)s64.size() * 64, (uint64_t)l128.size() * 128};
}

int main() {
    const size_t region = 1ull << 30;            // 1 GiB per kernel, 8 regions
    char *buf = nullptr;
    uint32_t *sink = nullptr;
    CHECK(hipMalloc(&buf, 8 * region));
    CHECK(hipMalloc(&sink, 64u << 20));
    CHECK(hipMemset(buf, 1, 8 * region));
    CHECK(hipDeviceSynchronize());
    const uint32_t n = 1u << 20;                 // gathers per kernel
    std::printf("[\n");
    // 0: coalesced stream of region 0 (1 GiB: also leaves the Infinity Cache
    // holding region 0, so every gather below starts cold)
    {
        const size_t nv = region / 16;
        hipLaunchKernelGGL(stream16, dim3(4096), dim3(BLOCK), 0, 0, (const uint4 *)buf, nv, sink);
        CHECK(hipDeviceSynchronize());
        std::printf(" {\"kernel\": \"stream16\", \"bytes\": %zu, \"sectors64\": %zu, \"lines128\": %zu},\n",
                    nv * 16, nv * 16, nv * 16);
    }
#define RUN(R, S, reg)                                                                               \
    {                                                                                                \
        const uint64_t nrec = (region / S) >= (1ull << 24) ? (1ull << 24) : (1ull << 22);             \
        const char *b = buf + (reg) * region;                                                        \
        hipLaunchKernelGGL((gather<R, S>), dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, 0, b, nrec, n, sink); \
        CHECK(hipDeviceSynchronize());                                                               \
        const Spans sp = spans((uint64_t)(reg) * region, nrec, n, R, S);                             \
        std::printf(" {\"kernel\": \"gather<%d, %d>\", \"bytes\": %llu, \"sectors64\": %llu, \"lines128\": %llu},\n", R, S, \
                    (unsigned long long)sp.bytes, (unsigned long long)sp.sectors64, (unsigned long long)sp.lines128); \
    }
    RUN(16, 16, 1)
    RUN(64, 64, 2)
    RUN(96, 96, 3)
    RUN(96, 128, 4)
    RUN(128, 128, 5)
    RUN(48, 48, 6)
    {
        const uint64_t nrec = 1ull << 22;
        const char *b = buf + 7 * region;
        hipLaunchKernelGGL(gather_bc<8>, dim3((8 * n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, 0, b, nrec, n, sink);
        CHECK(hipDeviceSynchronize());
        const Spans sp = spans(7 * region, nrec, n, 96, 96);
        std::printf(" {\"kernel\": \"gather_bc<8>\", \"bytes\": %llu, \"sectors64\": %llu, \"lines128\": %llu}\n",
                    (unsigned long long)sp.bytes, (unsigned long long)sp.sectors64, (unsigned long long)sp.lines128);
    }
    std::printf("]\n");
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
