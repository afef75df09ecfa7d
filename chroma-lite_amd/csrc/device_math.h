// device_math.h -- float3 algebra for the gfx950 kernels.
//
// Same value semantics as the reference's linalg.h/rotate.h (chroma/cuda/
// linalg.h:4-174, rotate.h:21-28); every multiply-add that nvcc contracts is an
// explicit fmaf, everything else is a separately rounded IEEE op
// (-ffp-contract=off), so results are bit-identical to the CPU oracle.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/chroma_fmath.h"

namespace chr {

constexpr float PI_F = 3.141592653589793f;   // physical_constants.h

struct V3 {
    float x, y, z;
};

__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ V3 operator*(V3 a, float c) { return v3(a.x * c, a.y * c, a.z * c); }
__device__ __forceinline__ V3 operator/(V3 a, float c) { return v3(a.x / c, a.y / c, a.z / c); }
// the rest of linalg.h's float3/float operators (self-test kernels, selftest.hip)
__device__ __forceinline__ V3 operator*(float c, V3 a) { return v3(c * a.x, c * a.y, c * a.z); }
__device__ __forceinline__ V3 operator/(float c, V3 a) { return v3(c / a.x, c / a.y, c / a.z); }
__device__ __forceinline__ V3 operator+(V3 a, float c) { return v3(a.x + c, a.y + c, a.z + c); }
__device__ __forceinline__ V3 operator+(float c, V3 a) { return v3(c + a.x, c + a.y, c + a.z); }
__device__ __forceinline__ V3 operator-(V3 a, float c) { return v3(a.x - c, a.y - c, a.z - c); }
__device__ __forceinline__ V3 operator-(float c, V3 a) { return v3(c - a.x, c - a.y, c - a.z); }
__device__ __forceinline__ V3 &operator+=(V3 &a, V3 b) { a = a + b; return a; }
__device__ __forceinline__ V3 &operator-=(V3 &a, V3 b) { a = a - b; return a; }
__device__ __forceinline__ V3 &operator+=(V3 &a, float c) { a = a + c; return a; }
__device__ __forceinline__ V3 &operator-=(V3 &a, float c) { a = a - c; return a; }
__device__ __forceinline__ V3 &operator*=(V3 &a, float c) { a = a * c; return a; }
__device__ __forceinline__ V3 &operator/=(V3 &a, float c) { a = a / c; return a; }

__device__ __forceinline__ float dot(V3 a, V3 b) { return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x)); }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return v3(__builtin_fmaf(a.y, b.z, -(a.z * b.y)), __builtin_fmaf(a.z, b.x, -(a.x * b.z)),
              __builtin_fmaf(a.x, b.y, -(a.y * b.x)));
}
__device__ __forceinline__ float norm(V3 a) { return __builtin_sqrtf(dot(a, a)); }
__device__ __forceinline__ V3 normalize(V3 a) { return a / norm(a); }
// p + d*v
__device__ __forceinline__ V3 axpy(float d, V3 v, V3 p) {
    return v3(__builtin_fmaf(d, v.x, p.x), __builtin_fmaf(d, v.y, p.y), __builtin_fmaf(d, v.z, p.z));
}
// IEEE fminf/fmaxf semantics (NaN loses), spelled out so both targets agree
__device__ __forceinline__ float fmin_(float a, float b) {
    if (chr_isnan(a)) return b;
    if (chr_isnan(b)) return a;
    return a < b ? a : b;
}
__device__ __forceinline__ float fmax_(float a, float b) {
    if (chr_isnan(a)) return b;
    if (chr_isnan(b)) return a;
    return a > b ? a : b;
}

// rotate a by phi about axis n (Rodrigues)
__device__ __forceinline__ V3 rotate(V3 a, float phi, V3 n) {
    float s, c;
    chr_sincosf(phi, &s, &c);
    const float d = dot(a, n);
    const float omc = 1.0f - c;
    const V3 cr = cross(a, n);
    return v3(__builtin_fmaf(cr.x, s, __builtin_fmaf(n.x * d, omc, a.x * c)),
              __builtin_fmaf(cr.y, s, __builtin_fmaf(n.y * d, omc, a.y * c)),
              __builtin_fmaf(cr.z, s, __builtin_fmaf(n.z * d, omc, a.z * c)));
}

}  // namespace chr
