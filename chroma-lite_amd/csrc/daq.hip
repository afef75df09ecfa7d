// daq.hip -- gfx950 DAQ kernels (the consumer of propagate's output) + C ABI.
//
// Reference: chroma/cuda/daq.cu (run_daq 35-83, run_daq_many 85-145,
// reset_earliest_time_int 25-33, convert_* 147-172) driven by GPUDaq
// (chroma/gpu/daq.py:37-101) with the Detector struct of detector.h:4-22.
//
// MI355X layout: the per-channel accumulators are three u32 arrays
// (ndaq*nchannels each; 29k channels = 116 KB, L2-resident), updated with
// device atomics whose results are order-independent (unsigned min of the
// time's bit pattern, integer charge sum, history OR).  A DAQ pass reads
// 20 B per photon (t, flags, last_hit, weight + the solid map entry of hit
// photons) and is HBM/launch bound; the chunked launches of the reference are
// folded into one launch in which work-item `slot` walks chunk positions
// slot, slot+cap, ... with its RNG state in registers (same draws, same order).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/chroma_amd.h"
#include "../../include/chroma_fmath.h"
#include "../../include/chroma_rng.h"
#include "common.h"

namespace chr_daq {

constexpr int BLOCK = 256;

// interpolate.h:32-58 (interp), as used by random.h:26-30 sample_cdf(x, y)
__device__ float interp(float x, int n, const float *xp, const float *fp) {
    int lower = 0, upper = n - 1;
    if (x <= xp[lower]) return fp[lower];
    if (x >= xp[upper]) return fp[upper];
    while (lower < upper - 1) {
        const int half = (lower + upper) / 2;
        if (x < xp[half]) upper = half; else lower = half;
    }
    const float df = fp[upper] - fp[lower];
    const float dx = xp[upper] - xp[lower];
    return fp[lower] + (df * (x - xp[lower])) / dx;
}

__device__ __forceinline__ float sample_cdf_xy(chr_xorwow &rng, int ncdf, const float *cdf_x, const float *cdf_y) {
    return interp(chr_uniform01(&rng), ncdf, cdf_y, cdf_x);
}

__device__ __forceinline__ void load_rng(const uint32_t *st, uint32_t ns, uint32_t s, chr_xorwow &r) {
    r.d = st[s]; r.v0 = st[ns + s]; r.v1 = st[2 * ns + s]; r.v2 = st[3 * ns + s]; r.v3 = st[4 * ns + s];
    r.v4 = st[5 * ns + s];
}
__device__ __forceinline__ void store_rng(uint32_t *st, uint32_t ns, uint32_t s, const chr_xorwow &r) {
    st[s] = r.d; st[ns + s] = r.v0; st[2 * ns + s] = r.v1; st[3 * ns + s] = r.v2; st[4 * ns + s] = r.v3;
    st[5 * ns + s] = r.v4;
}

struct DaqPhotons {
    const float *t, *weights;
    const uint32_t *flags;
    const int32_t *last_hit;
};

// daq.cu:25-33 + the zero fills of daq.py:56-60
__global__ __launch_bounds__(BLOCK) void begin_kernel(uint32_t *time_int, uint32_t *q_int, uint32_t *hist, uint32_t n,
                                                      uint32_t maxtime_bits) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    time_int[i] = maxtime_bits;
    q_int[i] = 0u;
    hist[i] = 0u;
}

// daq.cu:35-83 over all chunks of [start, start+n): slot loops over chunk positions
__global__ __launch_bounds__(BLOCK) void run_daq_kernel(uint32_t *rng_states, uint32_t nslots, uint32_t detection_state,
                                                        int32_t start, uint32_t n, uint32_t cap, DaqPhotons ph,
                                                        const uint32_t *solid_map, chr_daq_detector det,
                                                        uint32_t *time_int, uint32_t *q_int, uint32_t *hist,
                                                        float global_weight) {
    const uint32_t slot = blockIdx.x * BLOCK + threadIdx.x;
    if (slot >= cap || slot >= n) return;
    chr_xorwow rng;
    bool loaded = false;
    for (uint32_t pos = slot; pos < n; pos += cap) {
        const uint32_t photon_id = (uint32_t)start + pos;
        const int triangle_id = ph.last_hit[photon_id];
        if (triangle_id <= -1) continue;
        const int solid_id = (int)solid_map[triangle_id];
        const uint32_t history = ph.flags[photon_id];
        const int channel_index = det.d_solid_id_to_channel_index[solid_id];
        if (!(channel_index >= 0 && (history & detection_state))) continue;
        if (!loaded) { load_rng(rng_states, nslots, slot, rng); loaded = true; }
        const float weight = ph.weights[photon_id] * global_weight;
        if (chr_uniform01(&rng) < weight) {
            const float time = ph.t[photon_id] + sample_cdf_xy(rng, det.time_cdf_len, det.d_time_cdf_x, det.d_time_cdf_y);
            const float charge = sample_cdf_xy(rng, det.charge_cdf_len, det.d_charge_cdf_x, det.d_charge_cdf_y);
            const uint32_t charge_int = chr_sat_u32(__builtin_roundf(charge / det.charge_unit));
            atomicMin(time_int + channel_index, __float_as_uint(time));
            atomicAdd(q_int + channel_index, charge_int);
            atomicOr(hist + channel_index, history);
        }
    }
    if (loaded) store_rng(rng_states, nslots, slot, rng);
}

// daq.cu:85-145: one photon per workgroup of `ntpb` slots; workgroup b runs
// photons b, b+max_blocks, ... (the reference's successive chunks)
__global__ void run_daq_many_kernel(uint32_t *rng_states, uint32_t nslots, uint32_t *normal_cache,
                                    uint32_t detection_state, int32_t start, uint32_t n, uint32_t max_blocks,
                                    DaqPhotons ph, const uint32_t *solid_map, chr_daq_detector det,
                                    uint32_t *time_int, uint32_t *q_int, uint32_t *hist, int32_t ndaq,
                                    int32_t channel_stride, float global_weight) {
    const uint32_t b = blockIdx.x;
    const uint32_t slot = threadIdx.x + blockDim.x * b;
    chr_xorwow rng;
    uint32_t nflag = 0, nextra = 0;
    bool loaded = false;
    for (uint32_t pos = b; pos < n; pos += max_blocks) {
        const uint32_t photon_id = (uint32_t)start + pos;
        const int triangle_id = ph.last_hit[photon_id];
        // daq.cu:120-122; a wire-plane hit (-2) leaves the reference's shared
        // solid/channel words unset (UB): defined here as "not detected"
        if (triangle_id <= -1) continue;
        const int solid_id = (int)solid_map[triangle_id];
        const uint32_t history = ph.flags[photon_id];
        const int channel_index = det.d_solid_id_to_channel_index[solid_id];
        if (channel_index < 0 || !(history & detection_state)) continue;
        const float photon_time = ph.t[photon_id];
        const float weight = ph.weights[photon_id] * global_weight;
        if (!loaded) {
            load_rng(rng_states, nslots, slot, rng);
            nflag = normal_cache[slot];
            nextra = normal_cache[nslots + slot];
            loaded = true;
        }
        for (int i = (int)threadIdx.x; i < ndaq; i += (int)blockDim.x) {
            const int channel_offset = channel_index + i * channel_stride;
            if (chr_uniform01(&rng) < weight) {
                float time = photon_time + chr_normal(&rng, &nflag, &nextra);
                time = time + sample_cdf_xy(rng, det.time_cdf_len, det.d_time_cdf_x, det.d_time_cdf_y);
                const float charge = sample_cdf_xy(rng, det.charge_cdf_len, det.d_charge_cdf_x, det.d_charge_cdf_y);
                const uint32_t charge_int = chr_sat_u32(__builtin_roundf(charge / det.charge_unit));
                atomicMin(time_int + channel_offset, __float_as_uint(time));
                atomicAdd(q_int + channel_offset, charge_int);
                atomicOr(hist + channel_offset, history);
            }
        }
    }
    if (loaded) {
        store_rng(rng_states, nslots, slot, rng);
        normal_cache[slot] = nflag;
        normal_cache[nslots + slot] = nextra;
    }
}

// daq.cu:147-172
__global__ __launch_bounds__(BLOCK) void end_kernel(const uint32_t *time_int, float *time, const uint32_t *q_int,
                                                    float *q, uint32_t n, int32_t nchannels, float charge_unit) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    time[i] = __uint_as_float(time_int[i]);
    if ((int32_t)i < nchannels) q[i] = (float)q_int[i] * charge_unit;
}

// detected photons per channel (the selection of count_photon_hits,
// propagate.cu:172-199, histogrammed by channel): the per-rank array that the
// photon-sharded run reduces over RCCL
__global__ __launch_bounds__(BLOCK) void channel_counts_kernel(const uint32_t *flags, const int32_t *last_hit,
                                                               int32_t start, uint32_t n, uint32_t detection_state,
                                                               const uint32_t *solid_map, const int32_t *s2c,
                                                               int32_t nchannels, uint32_t *counts) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = (uint32_t)start + i;
    if (!(flags[p] & detection_state)) return;
    const int tri = last_hit[p];
    if (tri <= -1) return;
    const int c = s2c[solid_map[tri]];
    if (c >= 0 && c < nchannels) atomicAdd(counts + c, 1u);
}

inline unsigned grid_for(uint64_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

}  // namespace chr_daq

using namespace chr_daq;

extern "C" int chr_daq_begin(uint32_t *d_time_int, uint32_t *d_q_int, uint32_t *d_history, uint32_t n, float maxtime,
                             void *stream) {
    if (!d_time_int || !d_q_int || !d_history) return chr::fail(CHR_ERR_INVALID, "chr_daq_begin: null argument");
    if (n == 0) return CHR_OK;
    hipLaunchKernelGGL(begin_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, (hipStream_t)stream, d_time_int, d_q_int,
                       d_history, n, __builtin_bit_cast(uint32_t, maxtime));
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_daq_acquire(const chr_photons *ph, uint32_t *d_rng_states, uint32_t rng_nslots,
                               uint32_t *d_normal_cache, uint32_t detection_state, int32_t start_photon,
                               int32_t nphotons, const uint32_t *d_solid_map, const chr_daq_detector *det,
                               uint32_t *d_time_int, uint32_t *d_q_int, uint32_t *d_history, int32_t ndaq,
                               int32_t stride, float global_weight, int32_t ntpb, int32_t max_blocks, void *vstream) {
    if (!ph || !ph->d_t || !ph->d_flags || !ph->d_last_hit_triangles || !ph->d_weights || !d_rng_states ||
        !d_solid_map || !det || !det->d_solid_id_to_channel_index || !d_time_int || !d_q_int || !d_history)
        return chr::fail(CHR_ERR_INVALID, "chr_daq_acquire: null argument");
    if (!det->d_time_cdf_x || !det->d_time_cdf_y || !det->d_charge_cdf_x || !det->d_charge_cdf_y ||
        det->time_cdf_len < 2 || det->charge_cdf_len < 2)
        return chr::fail(CHR_ERR_INVALID, "chr_daq_acquire: time/charge CDFs missing");
    if (ndaq < 1 || ntpb <= 0 || max_blocks <= 0 || start_photon < 0)
        return chr::fail(CHR_ERR_INVALID, "chr_daq_acquire: bad ndaq / launch shape");
    if (nphotons <= 0) return CHR_OK;
    hipStream_t stream = (hipStream_t)vstream;
    DaqPhotons p{ph->d_t, ph->d_weights, ph->d_flags, ph->d_last_hit_triangles};
    if (ndaq == 1) {
        const uint64_t cap = (uint64_t)ntpb * max_blocks;
        if (cap > rng_nslots && (uint64_t)nphotons > rng_nslots)
            return chr::fail(CHR_ERR_INVALID, "chr_daq_acquire: %d photons per chunk but only %u rng states",
                             (int)std::min<uint64_t>(cap, nphotons), rng_nslots);
        const uint32_t threads = (uint32_t)std::min<uint64_t>(cap, (uint64_t)nphotons);
        hipLaunchKernelGGL(run_daq_kernel, dim3(grid_for(threads)), dim3(BLOCK), 0, stream, d_rng_states, rng_nslots,
                           detection_state, start_photon, (uint32_t)nphotons, (uint32_t)std::min<uint64_t>(cap, 0xFFFFFFFFu),
                           p, d_solid_map, *det, d_time_int, d_q_int, d_history, global_weight);
    } else {
        if (!d_normal_cache) return chr::fail(CHR_ERR_INVALID, "chr_daq_acquire: ndaq > 1 needs the normal cache");
        if (ntpb > 1024) return chr::fail(CHR_ERR_INVALID, "chr_daq_acquire: nthreads_per_block > 1024");
        const uint32_t blocks = (uint32_t)std::min<int64_t>(max_blocks, nphotons);
        if ((uint64_t)ntpb * blocks > rng_nslots)
            return chr::fail(CHR_ERR_INVALID, "chr_daq_acquire: %u slots needed, %u rng states",
                             (unsigned)(ntpb * blocks), rng_nslots);
        if (stride < 0) return chr::fail(CHR_ERR_INVALID, "chr_daq_acquire: negative stride");
        hipLaunchKernelGGL(run_daq_many_kernel, dim3(blocks), dim3(ntpb), 0, stream, d_rng_states, rng_nslots,
                           d_normal_cache, detection_state, start_photon, (uint32_t)nphotons, (uint32_t)max_blocks, p,
                           d_solid_map, *det, d_time_int, d_q_int, d_history, ndaq, stride, global_weight);
    }
    CHR_HIP_CHECK(hipGetLastError());
    CHR_HIP_CHECK(hipStreamSynchronize(stream));   // daq.py:91
    return CHR_OK;
}

extern "C" int chr_daq_end(const uint32_t *d_time_int, float *d_time, const uint32_t *d_q_int, float *d_q, uint32_t n,
                           int32_t nchannels, float charge_unit, void *stream) {
    if (!d_time_int || !d_time || !d_q_int || !d_q) return chr::fail(CHR_ERR_INVALID, "chr_daq_end: null argument");
    if (n == 0) return CHR_OK;
    hipLaunchKernelGGL(end_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, (hipStream_t)stream, d_time_int, d_time, d_q_int,
                       d_q, n, nchannels, charge_unit);
    CHR_HIP_CHECK(hipGetLastError());
    CHR_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    return CHR_OK;
}

extern "C" int chr_channel_hit_counts(const chr_photons *ph, int32_t start_photon, int32_t nphotons,
                                      uint32_t detection_state, const uint32_t *d_solid_map,
                                      const int32_t *d_solid_id_to_channel_index, uint32_t *d_counts,
                                      int32_t nchannels, void *stream) {
    if (!ph || !ph->d_flags || !ph->d_last_hit_triangles || !d_solid_map || !d_solid_id_to_channel_index || !d_counts)
        return chr::fail(CHR_ERR_INVALID, "chr_channel_hit_counts: null argument");
    if (nphotons <= 0 || nchannels <= 0) return CHR_OK;
    hipLaunchKernelGGL(channel_counts_kernel, dim3(grid_for((uint32_t)nphotons)), dim3(BLOCK), 0, (hipStream_t)stream,
                       ph->d_flags, ph->d_last_hit_triangles, start_photon, (uint32_t)nphotons, detection_state,
                       d_solid_map, d_solid_id_to_channel_index, nchannels, d_counts);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}
