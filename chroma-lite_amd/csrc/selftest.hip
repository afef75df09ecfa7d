// selftest.hip -- device self-test kernels: the reference's own unit-test
// kernels (test/linalg_test.cu, test/rotate_test.cu, test/test_sample_cdf.cu)
// run over THIS build's device math (device_math.h, sampling.h: the same
// functions the propagate kernels inline), so the reference's numpy / KS pins
// apply to the HIP path.  Exposed through the C ABI (chr_selftest_*) for
// tests only.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/chroma_amd.h"
#include "common.h"
#include "device_math.h"
#include "sampling.h"
#include "device_geometry.h"

namespace chr {
namespace {

constexpr int TB = 256;

__device__ __forceinline__ V3 ld3(const float *p, uint32_t i) { return v3(p[3 * i], p[3 * i + 1], p[3 * i + 2]); }
__device__ __forceinline__ void st3(float *p, uint32_t i, V3 v) { p[3 * i] = v.x; p[3 * i + 1] = v.y; p[3 * i + 2] = v.z; }

// test/linalg_test.cu: one kernel per operator, in the reference's order
__global__ __launch_bounds__(TB) void linalg_kernel(int op, uint32_t n, const float *A, const float *B, float c,
                                                    float *out) {
    const uint32_t i = blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    V3 a = ld3(A, i);
    const V3 b = ld3(B, i);
    switch (op) {
        case CHR_LINALG_FLOAT3ADD: st3(out, i, a + b); break;
        case CHR_LINALG_FLOAT3ADDEQUAL: a += b; st3(out, i, a); break;
        case CHR_LINALG_FLOAT3SUB: st3(out, i, a - b); break;
        case CHR_LINALG_FLOAT3SUBEQUAL: a -= b; st3(out, i, a); break;
        case CHR_LINALG_FLOAT3ADDFLOAT: st3(out, i, a + c); break;
        case CHR_LINALG_FLOAT3ADDFLOATEQUAL: a += c; st3(out, i, a); break;
        case CHR_LINALG_FLOATADDFLOAT3: st3(out, i, c + a); break;
        case CHR_LINALG_FLOAT3SUBFLOAT: st3(out, i, a - c); break;
        case CHR_LINALG_FLOAT3SUBFLOATEQUAL: a -= c; st3(out, i, a); break;
        case CHR_LINALG_FLOATSUBFLOAT3: st3(out, i, c - a); break;
        case CHR_LINALG_FLOAT3MULFLOAT: st3(out, i, a * c); break;
        case CHR_LINALG_FLOAT3MULFLOATEQUAL: a *= c; st3(out, i, a); break;
        case CHR_LINALG_FLOATMULFLOAT3: st3(out, i, c * a); break;
        case CHR_LINALG_FLOAT3DIVFLOAT: st3(out, i, a / c); break;
        case CHR_LINALG_FLOAT3DIVFLOATEQUAL: a /= c; st3(out, i, a); break;
        case CHR_LINALG_FLOATDIVFLOAT3: st3(out, i, c / a); break;
        case CHR_LINALG_DOT: out[i] = dot(a, b); break;
        case CHR_LINALG_CROSS: st3(out, i, cross(a, b)); break;
        case CHR_LINALG_NORM: out[i] = norm(a); break;
        case CHR_LINALG_MINUSFLOAT3: st3(out, i, -a); break;
        default: break;
    }
}

// test/rotate_test.cu
__global__ __launch_bounds__(TB) void rotate_kernel(uint32_t n, const float *A, const float *phi, V3 axis, float *out) {
    const uint32_t i = blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    st3(out, i, rotate(ld3(A, i), phi[i], axis));
}

// test/test_sample_cdf.cu: one draw per slot from its (curand_init-ed) state
__global__ __launch_bounds__(TB) void sample_cdf_kernel(uint32_t n, const uint32_t *states, uint32_t nslots, int ncdf,
                                                        const float *cdf_x, const float *cdf_y, float x0, float delta,
                                                        int uniform_grid, const uint32_t *index, float *out) {
    const uint32_t i = blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    chr_xorwow s;
    s.d = states[i]; s.v0 = states[nslots + i]; s.v1 = states[2 * nslots + i];
    s.v2 = states[3 * nslots + i]; s.v3 = states[4 * nslots + i]; s.v4 = states[5 * nslots + i];
    out[i] = uniform_grid == 2 ? sample_cdf_indexed(s, x0, delta, cdf_y, index, TIME_INDEX_BUCKETS)
             : uniform_grid  ? sample_cdf(s, ncdf, x0, delta, cdf_y)
                             : sample_cdf(s, ncdf, cdf_x, cdf_y);
}

inline unsigned blocks(uint32_t n) { return (n + TB - 1) / TB; }

}  // namespace
}  // namespace chr

extern "C" int chr_selftest_linalg(int32_t op, uint32_t n, const float *d_a, const float *d_b, float c, float *d_out,
                                   void *stream) {
    if (op < 0 || op >= CHR_LINALG_NOPS) return chr::fail(CHR_ERR_INVALID, "chr_selftest_linalg: unknown op %d", op);
    if (n == 0) return CHR_OK;
    if (!d_a || !d_b || !d_out) return chr::fail(CHR_ERR_INVALID, "chr_selftest_linalg: null argument");
    hipLaunchKernelGGL(chr::linalg_kernel, dim3(chr::blocks(n)), dim3(chr::TB), 0, (hipStream_t)stream, op, n, d_a, d_b,
                       c, d_out);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_selftest_rotate(uint32_t n, const float *d_a, const float *d_phi, float nx, float ny, float nz,
                                   float *d_out, void *stream) {
    if (n == 0) return CHR_OK;
    if (!d_a || !d_phi || !d_out) return chr::fail(CHR_ERR_INVALID, "chr_selftest_rotate: null argument");
    hipLaunchKernelGGL(chr::rotate_kernel, dim3(chr::blocks(n)), dim3(chr::TB), 0, (hipStream_t)stream, n, d_a, d_phi,
                       chr::V3{nx, ny, nz}, d_out);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_selftest_sample_cdf(uint32_t n, const uint32_t *d_states, uint32_t nslots, int32_t ncdf,
                                       const float *d_cdf_x, const float *d_cdf_y, float x0, float delta,
                                       int32_t uniform_grid, float *d_out, void *stream) {
    if (n == 0) return CHR_OK;
    if (!d_states || !d_cdf_y || !d_out || (!uniform_grid && !d_cdf_x) || n > nslots || ncdf < 2 || uniform_grid < 0 ||
        uniform_grid > 2)
        return chr::fail(CHR_ERR_INVALID, "chr_selftest_sample_cdf: bad argument");
    uint32_t *d_index = nullptr;
    if (uniform_grid == 2) {   // the geometry upload's bucket index of the CDF (synchronous)
        std::vector<float> h((size_t)ncdf);
        std::vector<uint32_t> idx;
        CHR_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
        CHR_HIP_CHECK(hipMemcpy(h.data(), d_cdf_y, h.size() * 4, hipMemcpyDeviceToHost));
        if (!chr::time_cdf_index(h.data(), 1, (uint32_t)ncdf, (uint32_t)ncdf, idx))
            return chr::fail(CHR_ERR_INVALID, "chr_selftest_sample_cdf: CDF not indexable (non-finite or decreasing)");
        CHR_HIP_CHECK(hipMalloc(&d_index, idx.size() * 4));
        CHR_HIP_CHECK(hipMemcpy(d_index, idx.data(), idx.size() * 4, hipMemcpyHostToDevice));
    }
    hipLaunchKernelGGL(chr::sample_cdf_kernel, dim3(chr::blocks(n)), dim3(chr::TB), 0, (hipStream_t)stream, n, d_states,
                       nslots, ncdf, d_cdf_x, d_cdf_y, x0, delta, uniform_grid, d_index, d_out);
    hipError_t e = hipGetLastError();
    if (d_index) {
        if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
        (void)hipFree(d_index);
    }
    if (e != hipSuccess) return chr::fail(CHR_ERR_HIP, "chr_selftest_sample_cdf: %s", hipGetErrorString(e));
    return CHR_OK;
}
