// pdf.hip -- gfx950 PDF / likelihood-support kernels (consumers of the DAQ
// output) + C ABI.
//
// Reference: chroma/cuda/pdf.cu (bin_hits 9-32, accumulate_bincount 34-96,
// accumulate_nearest_neighbor[_block] 98-219, accumulate_moments 223-266,
// accumulate_kernel_eval 271-368) driven by GPUPDF / GPUKernelPDF
// (chroma/gpu/pdf.py:7-372).
//
// All per-channel passes read a few words per channel (29k channels x ndaq
// DAQ copies) and are HBM/launch bound; one work-item per channel keeps the
// reference's serial accumulation order (float accumulators, as the
// reference) so the results are deterministic.  The nearest-neighbour pass
// replaces the reference's per-block serial insertion sort (piksrt, O(n^2) on
// one thread, 1000-entry table) with a rank selection spread over the block:
// each candidate distance counts the candidates that sort before it (value,
// then index) and the ones ranking below min_bin_content land in their sorted
// slot -- the same sorted prefix, for any table size.
//
// Defined reference edges: a charge below 0 converts to 0 (CUDA's saturating
// float->u32 conversion, made explicit); time / charge bins are clamped to
// the last bin of the channel (the reference can spill (t - tmin)/(tmax -
// tmin)*tbins == tbins into the next row); the moment / kernel passes cover
// the first len(hitcount) channel words (the reference indexes the per-channel
// accumulators with every DAQ copy when ndaq > 1, out of bounds).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/chroma_amd.h"
#include "../../include/chroma_fmath.h"
#include "common.h"

namespace chr_pdf {

constexpr int BLOCK = 256;
constexpr int NEAREST_BLOCK = 256;
constexpr int NEAREST_LDS = 8192;   // candidates staged in LDS (32 KB); larger tables read global
constexpr float INV_ROOT2 = 0.70710678118654746f;   // pdf.cu:268
constexpr float ROOT_PI_BY_2 = 1.2533141373155001f;  // pdf.cu:269

__device__ __forceinline__ uint32_t sat_u32(float x) { return chr_sat_u32(x); }   // NaN, negatives, -0 -> 0

// pdf.cu:9-32
__global__ __launch_bounds__(BLOCK) void bin_hits_kernel(int nchannels, const float *channel_q,
                                                         const float *channel_time, uint32_t *hitcount, int tbins,
                                                         float tmin, float tmax, int qbins, float qmin, float qmax,
                                                         uint32_t *pdf) {
    const int id = blockIdx.x * BLOCK + threadIdx.x;
    if (id >= nchannels) return;
    const float q = (float)sat_u32(channel_q[id]);
    const float t = channel_time[id];
    if (t < 1e8f && t >= tmin && t < tmax && q >= qmin && q < qmax) {
        hitcount[id] += 1u;
        const int tbin = min((int)((t - tmin) / (tmax - tmin) * (float)tbins), tbins - 1);
        const int qbin = min((int)((q - qmin) / (qmax - qmin) * (float)qbins), qbins - 1);
        pdf[(size_t)id * tbins * qbins + (size_t)tbin * qbins + qbin] += 1u;   // (channel, t, q) row major
    }
}

// pdf.cu:34-96: per channel, over the ndaq DAQ copies in order
__global__ __launch_bounds__(BLOCK) void bincount_kernel(int nchannels, int ndaq, const uint32_t *event_hit,
                                                         const float *event_time, const float *mc_time,
                                                         uint32_t *hitcount, uint32_t *bincount, float min_twidth,
                                                         float tmin, float tmax, int min_bin_content,
                                                         const uint32_t *map_channel_to_hit, uint32_t *work_queues) {
    const int c = blockIdx.x * BLOCK + threadIdx.x;
    if (c >= nchannels) return;
    float hc = (float)hitcount[c];
    float bc = (float)bincount[c];
    const float ev_t = event_time[c];
    const bool ev_hit = event_hit[c] != 0u;
    uint32_t *queue = ev_hit ? work_queues + (size_t)map_channel_to_hit[c] * (ndaq + 1) : nullptr;
    uint32_t next = ev_hit ? queue[0] : 0u;
    const double half_width = (double)min_twidth / 2.0;
    for (int i = 0; i < ndaq; i++) {
        const uint32_t off = (uint32_t)nchannels * i + c;
        const float mc = mc_time[off];
        if (mc >= 1e8f) continue;                  // not hit in this MC copy
        if (mc < tmin || mc > tmax) continue;      // outside the PDF range
        hc += 1.0f;
        if (!ev_hit) continue;
        if ((double)fabsf(mc - ev_t) < half_width) bc += 1.0f;
        if (bc < (float)min_bin_content) queue[next++] = off;
    }
    hitcount[c] = (uint32_t)hc;
    bincount[c] = (uint32_t)bc;
    if (ev_hit) queue[0] = next;
}

// pdf.cu:98-219: one block per hit channel.  Candidates = the stored table
// (up to its first entry > 1e8) followed by the queued MC distances; the
// min_bin_content smallest, ascending, replace the table's prefix.
__global__ __launch_bounds__(NEAREST_BLOCK) void nearest_kernel(int ndaq, const uint32_t *map_hit_to_channel,
                                                                const uint32_t *work_queues, const float *event_time,
                                                                const float *mc_time, float *nearest_mc, int k) {
    __shared__ float cand_lds[NEAREST_LDS];
    __shared__ float out_lds[NEAREST_LDS];
    __shared__ int table_len;
    const int hit = blockIdx.x;
    const uint32_t *queue = work_queues + (size_t)hit * (ndaq + 1);
    const int nq = (int)queue[0] - 1;
    const float ev_t = event_time[map_hit_to_channel[hit]];
    float *table = nearest_mc + (size_t)hit * k;
    if (threadIdx.x == 0) table_len = k;
    __syncthreads();
    for (int i = threadIdx.x; i < k; i += NEAREST_BLOCK)
        if (table[i] > 1e8f) atomicMin(&table_len, i);
    __syncthreads();
    const int nt = table_len;
    const int n = nt + nq;
    const bool staged = n <= NEAREST_LDS;
    auto value = [&](int j) -> float {
        return j < nt ? table[j] : fabsf(mc_time[queue[1 + j - nt]] - ev_t);
    };
    if (staged) {
        for (int j = threadIdx.x; j < n; j += NEAREST_BLOCK) cand_lds[j] = value(j);
        __syncthreads();
    }
    // total order: ascending, NaN after every number (all NaNs tie), ties by
    // position -- every rank below min(n, k) is taken exactly once
    for (int i = threadIdx.x; i < n; i += NEAREST_BLOCK) {
        const float v = staged ? cand_lds[i] : value(i);
        const bool vnan = v != v;
        int rank = 0;
        for (int j = 0; j < n && rank < k; j++) {
            const float w = staged ? cand_lds[j] : value(j);
            const bool wnan = w != w;
            const bool before = vnan ? !wnan : (w < v);
            const bool tie = vnan ? wnan : (w == v);
            rank += before || (tie && j < i);
        }
        if (rank < k) out_lds[rank] = v;
    }
    __syncthreads();
    const int m = min(n, k);
    for (int i = threadIdx.x; i < m; i += NEAREST_BLOCK) table[i] = out_lds[i];
}

// pdf.cu:223-266
__global__ __launch_bounds__(BLOCK) void moments_kernel(int time_only, int nchannels, const float *mc_time,
                                                        const float *mc_charge, float tmin, float tmax, float qmin,
                                                        float qmax, uint32_t *mom0, float *t_mom1, float *t_mom2,
                                                        float *q_mom1, float *q_mom2) {
    const int id = blockIdx.x * BLOCK + threadIdx.x;
    if (id >= nchannels) return;
    const float t = mc_time[id];
    if (time_only) {
        if (t < tmin || t > tmax) return;
    } else {
        const float q = mc_charge[id];
        if (t < tmin || t > tmax || q < qmin || q > qmax) return;
        q_mom1[id] += q;
        q_mom2[id] = fmaf(q, q, q_mom2[id]);       // nvcc contracts a*b + c
    }
    mom0[id] += 1u;
    t_mom1[id] += t;
    t_mom2[id] = fmaf(t, t, t_mom2[id]);
}

// Gaussian kernel normalised to [lo, hi] (pdf.cu:311-318 / 342-347 / 357-362)
__device__ __forceinline__ float window_norm(float lo, float hi, float mc, float inv_bw) {
    if (!(inv_bw > 0.0f)) return hi - lo;
    const float loarg = (lo - mc) * inv_bw * INV_ROOT2;
    const float hiarg = (hi - mc) * inv_bw * INV_ROOT2;
    return (chr_erff(hiarg) - chr_erff(loarg)) * ROOT_PI_BY_2;
}

// pdf.cu:271-368
__global__ __launch_bounds__(BLOCK) void kernel_eval_kernel(int time_only, int nchannels, const uint32_t *event_hit,
                                                            const float *event_time, const float *event_charge,
                                                            const float *mc_time, const float *mc_charge, float tmin,
                                                            float tmax, float qmin, float qmax, const float *inv_tbw,
                                                            const float *inv_qbw, uint32_t *hitcount,
                                                            float *time_pdf, float *charge_pdf) {
    const int id = blockIdx.x * BLOCK + threadIdx.x;
    if (id >= nchannels) return;
    const float t = mc_time[id];
    if (time_only) {
        if (t < tmin || t > tmax) return;
        hitcount[id] += 1u;
        if (!event_hit[id]) return;
        const float ibw = inv_tbw[id];
        const float arg = (t - event_time[id]) * ibw;
        const float term = chr_expf(-0.5f * arg * arg) * ibw;
        time_pdf[id] += term / window_norm(tmin, tmax, t, ibw);
    } else {
        const float q = mc_charge[id];
        if (t < tmin || t > tmax || q < qmin || q > qmax) return;
        hitcount[id] += 1u;
        if (!event_hit[id]) return;
        const float ibt = inv_tbw[id];
        const float at = (t - event_time[id]) * ibt;
        time_pdf[id] += chr_expf(-0.5f * at * at) / window_norm(tmin, tmax, t, ibt);
        const float ibq = inv_qbw[id];
        const float aq = (q - event_charge[id]) * ibq;
        charge_pdf[id] += chr_expf(-0.5f * aq * aq) / window_norm(qmin, qmax, q, ibq);
    }
}

inline unsigned grid_for(int64_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

}  // namespace chr_pdf

using namespace chr_pdf;

extern "C" int chr_pdf_bin_hits(int32_t nchannels, const float *d_channel_q, const float *d_channel_time,
                                uint32_t *d_hitcount, int32_t tbins, float tmin, float tmax, int32_t qbins, float qmin,
                                float qmax, uint32_t *d_pdf, void *stream) {
    if (!d_channel_q || !d_channel_time || !d_hitcount || !d_pdf)
        return chr::fail(CHR_ERR_INVALID, "chr_pdf_bin_hits: null argument");
    if (tbins <= 0 || qbins <= 0 || !(tmax > tmin) || !(qmax > qmin))
        return chr::fail(CHR_ERR_INVALID, "chr_pdf_bin_hits: empty binning");
    if (nchannels <= 0) return CHR_OK;
    hipLaunchKernelGGL(bin_hits_kernel, dim3(grid_for(nchannels)), dim3(BLOCK), 0, (hipStream_t)stream, nchannels,
                       d_channel_q, d_channel_time, d_hitcount, tbins, tmin, tmax, qbins, qmin, qmax, d_pdf);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_pdf_accumulate_bincount(int32_t nchannels, int32_t ndaq, const uint32_t *d_event_hit,
                                           const float *d_event_time, const float *d_mc_time, uint32_t *d_hitcount,
                                           uint32_t *d_bincount, float min_twidth, float tmin, float tmax,
                                           int32_t min_bin_content, const uint32_t *d_map_channel_to_hit,
                                           uint32_t *d_work_queues, void *stream) {
    if (!d_event_hit || !d_event_time || !d_mc_time || !d_hitcount || !d_bincount || !d_map_channel_to_hit)
        return chr::fail(CHR_ERR_INVALID, "chr_pdf_accumulate_bincount: null argument");
    if (ndaq < 1) return chr::fail(CHR_ERR_INVALID, "chr_pdf_accumulate_bincount: ndaq < 1");
    if (nchannels <= 0) return CHR_OK;
    hipLaunchKernelGGL(bincount_kernel, dim3(grid_for(nchannels)), dim3(BLOCK), 0, (hipStream_t)stream, nchannels,
                       ndaq, d_event_hit, d_event_time, d_mc_time, d_hitcount, d_bincount, min_twidth, tmin, tmax,
                       min_bin_content, d_map_channel_to_hit, d_work_queues);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_pdf_accumulate_nearest(int32_t nhit, int32_t ndaq, const uint32_t *d_map_hit_to_channel,
                                          const uint32_t *d_work_queues, const float *d_event_time,
                                          const float *d_mc_time, float *d_nearest_mc, int32_t min_bin_content,
                                          void *stream) {
    if (min_bin_content < 1 || min_bin_content > NEAREST_LDS)
        return chr::fail(CHR_ERR_INVALID, "chr_pdf_accumulate_nearest: min_bin_content must be in [1, %d]",
                         NEAREST_LDS);
    if (nhit <= 0) return CHR_OK;
    if (!d_map_hit_to_channel || !d_work_queues || !d_event_time || !d_mc_time || !d_nearest_mc)
        return chr::fail(CHR_ERR_INVALID, "chr_pdf_accumulate_nearest: null argument");
    if (ndaq < 1) return chr::fail(CHR_ERR_INVALID, "chr_pdf_accumulate_nearest: ndaq < 1");
    hipLaunchKernelGGL(nearest_kernel, dim3(nhit), dim3(NEAREST_BLOCK), 0, (hipStream_t)stream, ndaq,
                       d_map_hit_to_channel, d_work_queues, d_event_time, d_mc_time, d_nearest_mc, min_bin_content);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_pdf_accumulate_moments(int32_t time_only, int32_t nchannels, const float *d_mc_time,
                                          const float *d_mc_charge, float tmin, float tmax, float qmin, float qmax,
                                          uint32_t *d_mom0, float *d_t_mom1, float *d_t_mom2, float *d_q_mom1,
                                          float *d_q_mom2, void *stream) {
    if (!d_mc_time || !d_mom0 || !d_t_mom1 || !d_t_mom2 ||
        (!time_only && (!d_mc_charge || !d_q_mom1 || !d_q_mom2)))
        return chr::fail(CHR_ERR_INVALID, "chr_pdf_accumulate_moments: null argument");
    if (nchannels <= 0) return CHR_OK;
    hipLaunchKernelGGL(moments_kernel, dim3(grid_for(nchannels)), dim3(BLOCK), 0, (hipStream_t)stream, time_only,
                       nchannels, d_mc_time, d_mc_charge, tmin, tmax, qmin, qmax, d_mom0, d_t_mom1, d_t_mom2,
                       d_q_mom1, d_q_mom2);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_pdf_accumulate_kernel_eval(int32_t time_only, int32_t nchannels, const uint32_t *d_event_hit,
                                              const float *d_event_time, const float *d_event_charge,
                                              const float *d_mc_time, const float *d_mc_charge, float tmin,
                                              float tmax, float qmin, float qmax, const float *d_inv_time_bw,
                                              const float *d_inv_charge_bw, uint32_t *d_hitcount,
                                              float *d_time_pdf, float *d_charge_pdf, void *stream) {
    if (!d_event_hit || !d_event_time || !d_mc_time || !d_inv_time_bw || !d_hitcount || !d_time_pdf ||
        (!time_only && (!d_event_charge || !d_mc_charge || !d_inv_charge_bw || !d_charge_pdf)))
        return chr::fail(CHR_ERR_INVALID, "chr_pdf_accumulate_kernel_eval: null argument");
    if (nchannels <= 0) return CHR_OK;
    hipLaunchKernelGGL(kernel_eval_kernel, dim3(grid_for(nchannels)), dim3(BLOCK), 0, (hipStream_t)stream, time_only,
                       nchannels, d_event_hit, d_event_time, d_event_charge, d_mc_time, d_mc_charge, tmin, tmax, qmin,
                       qmax, d_inv_time_bw, d_inv_charge_bw, d_hitcount, d_time_pdf, d_charge_pdf);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}
