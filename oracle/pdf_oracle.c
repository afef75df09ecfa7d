/* pdf_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Sequential CPU restatement of the reference's PDF kernels
 * (chroma/cuda/pdf.cu), the checker for csrc/pdf.hip.  Only tests/ load it.
 * Each function loops over channels in index order and does exactly what one
 * reference thread does for that channel (float accumulators, the same
 * comparisons, the same multiply-add contractions spelled as fmaf).  The
 * defined edges of the HIP path are restated too (saturating charge
 * conversion, bins clamped to the channel's last bin).  erff/expf come from
 * include/chroma_fmath.h, shared with the kernels; parity of those two with
 * CUDA's fast-math erff/expf is unpinned (PDF section).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/chroma_fmath.h"

static uint32_t sat_u32(float x) {
    if (!(x > 0.0f)) return 0u;
    if (x >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)x;
}

/* pdf.cu:9-32 */
void orc_pdf_bin_hits(int nchannels, const float *channel_q, const float *channel_time, uint32_t *hitcount,
                      int tbins, float tmin, float tmax, int qbins, float qmin, float qmax, uint32_t *pdf) {
    for (int id = 0; id < nchannels; id++) {
        const float q = (float)sat_u32(channel_q[id]);
        const float t = channel_time[id];
        if (!(t < 1e8f && t >= tmin && t < tmax && q >= qmin && q < qmax)) continue;
        hitcount[id] += 1u;
        int tbin = (int)((t - tmin) / (tmax - tmin) * (float)tbins);
        int qbin = (int)((q - qmin) / (qmax - qmin) * (float)qbins);
        if (tbin > tbins - 1) tbin = tbins - 1;
        if (qbin > qbins - 1) qbin = qbins - 1;
        pdf[(size_t)id * tbins * qbins + (size_t)tbin * qbins + qbin] += 1u;
    }
}

/* pdf.cu:34-96 */
void orc_pdf_accumulate_bincount(int nchannels, int ndaq, const uint32_t *event_hit, const float *event_time,
                                 const float *mc_time, uint32_t *hitcount, uint32_t *bincount, float min_twidth,
                                 float tmin, float tmax, int min_bin_content, const uint32_t *map_channel_to_hit,
                                 uint32_t *work_queues) {
    for (int c = 0; c < nchannels; c++) {
        float hc = (float)hitcount[c], bc = (float)bincount[c];
        const int ev_hit = event_hit[c] != 0u;
        uint32_t *queue = ev_hit ? work_queues + (size_t)map_channel_to_hit[c] * (ndaq + 1) : NULL;
        uint32_t next = ev_hit ? queue[0] : 0u;
        for (int i = 0; i < ndaq; i++) {
            const uint32_t off = (uint32_t)nchannels * i + c;
            const float mc = mc_time[off];
            if (mc >= 1e8f) continue;
            if (mc < tmin || mc > tmax) continue;
            hc += 1.0f;
            if (!ev_hit) continue;
            if ((double)fabsf(mc - event_time[c]) < (double)min_twidth / 2.0) bc += 1.0f;
            if (bc < (float)min_bin_content) queue[next++] = off;
        }
        hitcount[c] = (uint32_t)hc;
        bincount[c] = (uint32_t)bc;
        if (ev_hit) queue[0] = next;
    }
}

/* ascending, NaN after every number (the HIP kernel's total order) */
static int cmp_float(const void *a, const void *b) {
    const float x = *(const float *)a, y = *(const float *)b;
    const int xn = x != x, yn = y != y;
    if (xn || yn) return xn - yn;
    return (x > y) - (x < y);
}

/* pdf.cu:98-150 (accumulate_nearest_neighbor: load table, append, piksrt, copy back) */
void orc_pdf_accumulate_nearest(int nhit, int ndaq, const uint32_t *map_hit_to_channel, const uint32_t *work_queues,
                                const float *event_time, const float *mc_time, float *nearest_mc, int k) {
    for (int h = 0; h < nhit; h++) {
        const uint32_t *queue = work_queues + (size_t)h * (ndaq + 1);
        const int nq = (int)queue[0] - 1;
        const float ev_t = event_time[map_hit_to_channel[h]];
        float *table = nearest_mc + (size_t)h * k;
        float *d = (float *)malloc(sizeof(float) * (size_t)(k + nq + 1));
        int n = 0;
        for (int i = 0; i < k; i++) {
            if (table[i] > 1e8f) break;
            d[n++] = table[i];
        }
        for (int i = 0; i < nq; i++) d[n++] = fabsf(mc_time[queue[i + 1]] - ev_t);
        qsort(d, (size_t)n, sizeof(float), cmp_float);
        for (int i = 0; i < n && i < k; i++) table[i] = d[i];
        free(d);
    }
}

/* pdf.cu:223-266 */
void orc_pdf_accumulate_moments(int time_only, int nchannels, const float *mc_time, const float *mc_charge,
                                float tmin, float tmax, float qmin, float qmax, uint32_t *mom0, float *t_mom1,
                                float *t_mom2, float *q_mom1, float *q_mom2) {
    for (int id = 0; id < nchannels; id++) {
        const float t = mc_time[id];
        if (time_only) {
            if (t < tmin || t > tmax) continue;
        } else {
            const float q = mc_charge[id];
            if (t < tmin || t > tmax || q < qmin || q > qmax) continue;
            q_mom1[id] += q;
            q_mom2[id] = chr_fmaf(q, q, q_mom2[id]);
        }
        mom0[id] += 1u;
        t_mom1[id] += t;
        t_mom2[id] = chr_fmaf(t, t, t_mom2[id]);
    }
}

static float window_norm(float lo, float hi, float mc, float inv_bw) {
    if (!(inv_bw > 0.0f)) return hi - lo;
    const float loarg = (lo - mc) * inv_bw * 0.70710678118654746f;
    const float hiarg = (hi - mc) * inv_bw * 0.70710678118654746f;
    return (chr_erff(hiarg) - chr_erff(loarg)) * 1.2533141373155001f;
}

/* pdf.cu:271-368 */
void orc_pdf_accumulate_kernel_eval(int time_only, int nchannels, const uint32_t *event_hit, const float *event_time,
                                    const float *event_charge, const float *mc_time, const float *mc_charge,
                                    float tmin, float tmax, float qmin, float qmax, const float *inv_tbw,
                                    const float *inv_qbw, uint32_t *hitcount, float *time_pdf, float *charge_pdf) {
    for (int id = 0; id < nchannels; id++) {
        const float t = mc_time[id];
        if (time_only) {
            if (t < tmin || t > tmax) continue;
            hitcount[id] += 1u;
            if (!event_hit[id]) continue;
            const float ibw = inv_tbw[id];
            const float arg = (t - event_time[id]) * ibw;
            const float term = chr_expf(-0.5f * arg * arg) * ibw;
            time_pdf[id] += term / window_norm(tmin, tmax, t, ibw);
        } else {
            const float q = mc_charge[id];
            if (t < tmin || t > tmax || q < qmin || q > qmax) continue;
            hitcount[id] += 1u;
            if (!event_hit[id]) continue;
            const float ibt = inv_tbw[id];
            const float at = (t - event_time[id]) * ibt;
            time_pdf[id] += chr_expf(-0.5f * at * at) / window_norm(tmin, tmax, t, ibt);
            const float ibq = inv_qbw[id];
            const float aq = (q - event_charge[id]) * ibq;
            charge_pdf[id] += chr_expf(-0.5f * aq * aq) / window_norm(qmin, qmax, q, ibq);
        }
    }
}

/* chr_erff over an array (math test) */
void orc_erff(int n, const float *x, float *y) {
    for (int i = 0; i < n; i++) y[i] = chr_erff(x[i]);
}
