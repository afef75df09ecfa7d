// sampling.h -- random sampling and table interpolation of the reference's
// random.h / interpolate.h, for the gfx950 kernels (propagate.hip) and their
// self-test kernels (selftest.hip).  Same operation order as the reference
// (chroma/cuda/random.h:9-55, interpolate.h:4-58); the a + b*c forms nvcc
// contracts are explicit fmaf; everything else is a separately rounded IEEE op.
#pragma once

#include "../../include/chroma_rng.h"
#include "device_math.h"

namespace chr {

// interpolate.h:4-29 (the 1.0* promotes the fraction to double)
__device__ __forceinline__ float interp_idx(float x, int n, const float *xp) {
    int lower = 0, upper = n - 1;
    if (x <= xp[lower]) return (float)lower;
    if (x >= xp[upper]) return (float)upper;
    while (lower < upper - 1) {
        int half = (lower + upper) / 2;
        if (x < xp[half]) upper = half; else lower = half;
    }
    float dx = xp[upper] - xp[lower];
    return (float)((double)lower + (double)(x - xp[lower]) / (double)dx);
}

// interpolate.h:32-58
__device__ __forceinline__ float interp(float x, int n, const float *xp, const float *fp) {
    int lower = 0, upper = n - 1;
    if (x <= xp[lower]) return fp[lower];
    if (x >= xp[upper]) return fp[upper];
    while (lower < upper - 1) {
        int half = (lower + upper) / 2;
        if (x < xp[half]) upper = half; else lower = half;
    }
    const float df = fp[upper] - fp[lower];
    const float dx = xp[upper] - xp[lower];
    return fp[lower] + (df * (x - xp[lower])) / dx;
}

// random.h:15-23
__device__ __forceinline__ V3 uniform_sphere(chr_xorwow &s) {
    const float theta = chr_uniform(&s, 0.0f, 2 * PI_F);
    const float u = chr_uniform(&s, -1.0f, 1.0f);
    const float c = chr_sqrtf(__builtin_fmaf(-u, u, 1.0f));
    float st, ct;
    chr_sincosf(theta, &st, &ct);
    return v3(c * ct, c * st, u);
}

// random.h:27-31: sample a tabulated CDF (cdf_y ascending from 0 to 1)
__device__ __forceinline__ float sample_cdf(chr_xorwow &rng, int ncdf, const float *cdf_x, const float *cdf_y) {
    return interp(chr_uniform01(&rng), ncdf, cdf_y, cdf_x);
}

// random.h:34-55: sample a CDF tabulated on the uniform grid x0 + delta*i
__device__ float sample_cdf(chr_xorwow &rng, int ncdf, float x0, float delta, const float *cdf_y) {
    const float u = chr_uniform01(&rng);
    int lower = 0, upper = ncdf - 1;
    while (lower < upper - 1) {
        int half = (lower + upper) / 2;
        if (u < cdf_y[half]) upper = half; else lower = half;
    }
    const float dcy = cdf_y[upper] - cdf_y[lower];
    return __builtin_fmaf(delta, (float)lower, x0) + (delta * (u - cdf_y[lower])) / dcy;
}

// random.h:34-55 over a non-decreasing CDF of >= 2 entries with a bucket index
// (index[b] = the largest j with cdf_y[j] <= b/nb clamped to [0, ncdf-2], nb a
// power of two; geometry.cpp time_cdf_index).  The reference's bisection ends on
// lower = the largest j with cdf_y[j] <= u clamped to [0, ncdf-2]; u lies in
// [b/nb, (b+1)/nb] for b = min(floor(u*nb), nb-1), so that j lies in
// [index[b], index[b+1]] and a bisection of that range finds the same lower: the
// same sample, from ~log2(ncdf/nb) probes instead of log2(ncdf).
__device__ float sample_cdf_indexed(chr_xorwow &rng, float x0, float delta, const float *cdf_y,
                                    const uint32_t *index, uint32_t nb) {
    const float u = chr_uniform01(&rng);
    const uint32_t b = min((uint32_t)(u * (float)nb), nb - 1u);
    int lower = (int)index[b], upper = (int)index[b + 1];
    while (lower < upper) {                 // the largest j in [lower, upper] with cdf_y[j] <= u, else lower
        const int half = (lower + upper + 1) >> 1;
        if (cdf_y[half] <= u) lower = half; else upper = half - 1;
    }
    const float dcy = cdf_y[lower + 1] - cdf_y[lower];
    return __builtin_fmaf(delta, (float)lower, x0) + (delta * (u - cdf_y[lower])) / dcy;
}

}  // namespace chr
