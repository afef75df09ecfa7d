/* chroma_rng.h -- cuRAND-XORWOW-compatible generator (state in registers).
 *
 * The reference draws every random number through cuRAND's default generator
 * (curandState = XORWOW; chroma/cuda/random.h:4-23, initialised by
 * curand_init(seed, id, 0) in chroma/gpu/tools.py:117-145).  cuRAND is not part
 * of ROCm, so the generator is restated here (Marsaglia xorwow, 2003):
 *
 *   curand_init(seed, subseq, offset):
 *     s0 = lo32(seed) ^ 0xaad26b49, s1 = hi32(seed) ^ 0xf7dcefdd
 *     t0 = 1099087573 * s0,          t1 = 2591861531 * s1
 *     d = 6615241 + t1 + t0
 *     v = {123456789 + t0, 362436069 ^ t0, 521288629 + t1, 88675123 ^ t1, 5783321 + t0}
 *     v <- A^(subseq * 2^67) v          (d is unchanged: 2^67 = 0 mod 2^32)
 *     v <- A^offset v, d += 362437 * offset
 *   curand():  t = v0 ^ (v0 >> 2); shift v; v4 = (v4 ^ (v4 << 4)) ^ (t ^ (t << 1));
 *              d += 362437; return v4 + d
 *   curand_uniform() = (float)x * 2^-32 + 2^-33        (range (0, 1])
 *
 * The recurrence and the 2^67 subsequence spacing are identical to rocRAND's
 * xorwow (/opt/rocm/include/rocrand/rocrand_xorwow.h:165-177, whose precomputed
 * sequence-jump table pins our jump-matrix construction in tests/); only the
 * seed salts differ (rocrand_xorwow.h:113-122), and those salts are the part
 * that is "parity unpinned" (no cuRAND in this image).
 *
 * A state is 6 x u32 {d, v0..v4}.  In HBM it is stored SoA: word k of slot s at
 * state[k * nslots + s], so a wave's state load is six 256-byte coalesced rows.
 */
#ifndef CHROMA_RNG_H
#define CHROMA_RNG_H

#include "chroma_fmath.h"

#if defined(__HIPCC__)
#define CHR_HOST_FN __host__ static inline
#else
#define CHR_HOST_FN static inline
#endif

typedef struct { uint32_t d, v0, v1, v2, v3, v4; } chr_xorwow;

CHR_FN uint32_t chr_xorwow_next(chr_xorwow *s) {
    uint32_t t = s->v0 ^ (s->v0 >> 2);
    s->v0 = s->v1; s->v1 = s->v2; s->v2 = s->v3; s->v3 = s->v4;
    s->v4 = (s->v4 ^ (s->v4 << 4)) ^ (t ^ (t << 1));
    s->d += 362437u;
    return s->v4 + s->d;
}

/* curand_uniform: x * 2^-32 + 2^-33 (the product is exact, so fused or not is identical) */
CHR_FN float chr_uniform01(chr_xorwow *s) {
    return (float)chr_xorwow_next(s) * 2.3283064365386963e-10f + 1.1641532182693481e-10f;
}

/* reference random.h:9-12: low + u*(high-low) */
CHR_FN float chr_uniform(chr_xorwow *s, float low, float high) {
    return low + chr_uniform01(s) * (high - low);
}

/* seed scrambling part of curand_init (before the subsequence jump) */
CHR_FN void chr_xorwow_seed(chr_xorwow *s, unsigned long long seed) {
    uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    s->d = 6615241u + t1 + t0;
    s->v0 = 123456789u + t0;
    s->v1 = 362436069u ^ t0;
    s->v2 = 521288629u + t1;
    s->v3 = 88675123u ^ t1;
    s->v4 = 5783321u + t0;
}

/* ---- GF(2) jump matrices.  A matrix is 160 columns x 5 words: col[b*5 + k] is
 * word k of the image of basis bit b (b = 32*word + bit), the layout rocRAND
 * uses for its precomputed tables. */
#define CHR_XW_MATWORDS 800

CHR_FN void chr_xw_matvec(const uint32_t *m, uint32_t v[5]) {
    uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
    for (int i = 0; i < 5; ++i) {
        uint32_t w = v[i];
        for (int j = 0; j < 32; ++j) {
            uint32_t b = 0u - ((w >> j) & 1u);
            const uint32_t *c = m + (i * 32 + j) * 5;
            r0 ^= b & c[0]; r1 ^= b & c[1]; r2 ^= b & c[2]; r3 ^= b & c[3]; r4 ^= b & c[4];
        }
    }
    v[0] = r0; v[1] = r1; v[2] = r2; v[3] = r3; v[4] = r4;
}

/* out = a o b (apply b first).  out must not alias a or b. */
CHR_HOST_FN void chr_xw_matmul(const uint32_t *a, const uint32_t *b, uint32_t *out) {
    for (int col = 0; col < 160; ++col) {
        uint32_t v[5];
        for (int k = 0; k < 5; ++k) v[k] = b[col * 5 + k];
        chr_xw_matvec(a, v);
        for (int k = 0; k < 5; ++k) out[col * 5 + k] = v[k];
    }
}

/* one-step transition matrix of the xorshift part */
CHR_HOST_FN void chr_xw_step_matrix(uint32_t *m) {
    for (int col = 0; col < 160; ++col) {
        uint32_t x[5] = {0, 0, 0, 0, 0};
        x[col / 32] = 1u << (col % 32);
        uint32_t t = x[0] ^ (x[0] >> 2);
        uint32_t y[5] = {x[1], x[2], x[3], x[4], (x[4] ^ (x[4] << 4)) ^ (t ^ (t << 1))};
        for (int k = 0; k < 5; ++k) m[col * 5 + k] = y[k];
    }
}

/* seq[i] = A^(2^(67+i)), i = 0..nlevels-1; caller provides nlevels*800 words. */
CHR_HOST_FN void chr_xw_sequence_matrices(uint32_t *seq, int nlevels) {
    uint32_t cur[CHR_XW_MATWORDS], tmp[CHR_XW_MATWORDS];
    chr_xw_step_matrix(cur);
    for (int i = 0; i < 67; ++i) { chr_xw_matmul(cur, cur, tmp); for (int k = 0; k < CHR_XW_MATWORDS; ++k) cur[k] = tmp[k]; }
    for (int l = 0; l < nlevels; ++l) {
        for (int k = 0; k < CHR_XW_MATWORDS; ++k) seq[l * CHR_XW_MATWORDS + k] = cur[k];
        chr_xw_matmul(cur, cur, tmp);
        for (int k = 0; k < CHR_XW_MATWORDS; ++k) cur[k] = tmp[k];
    }
}

/* off[i] = A^(2^i), i = 0..nlevels-1 */
CHR_HOST_FN void chr_xw_offset_matrices(uint32_t *off, int nlevels) {
    uint32_t cur[CHR_XW_MATWORDS], tmp[CHR_XW_MATWORDS];
    chr_xw_step_matrix(cur);
    for (int l = 0; l < nlevels; ++l) {
        for (int k = 0; k < CHR_XW_MATWORDS; ++k) off[l * CHR_XW_MATWORDS + k] = cur[k];
        chr_xw_matmul(cur, cur, tmp);
        for (int k = 0; k < CHR_XW_MATWORDS; ++k) cur[k] = tmp[k];
    }
}

/* curand_init(seed, subseq, offset) given precomputed jump tables
 * (seq: A^(2^(67+i)) for i < nseq; off: A^(2^i) for i < noff). */
CHR_FN void chr_xorwow_init(chr_xorwow *s, unsigned long long seed, unsigned long long subseq,
                            unsigned long long offset, const uint32_t *seq, int nseq,
                            const uint32_t *off, int noff) {
    chr_xorwow_seed(s, seed);
    uint32_t v[5] = {s->v0, s->v1, s->v2, s->v3, s->v4};
    for (int i = 0; i < nseq && subseq; ++i, subseq >>= 1)
        if (subseq & 1ull) chr_xw_matvec(seq + i * CHR_XW_MATWORDS, v);
    unsigned long long o = offset;
    for (int i = 0; i < noff && o; ++i, o >>= 1)
        if (o & 1ull) chr_xw_matvec(off + i * CHR_XW_MATWORDS, v);
    s->v0 = v[0]; s->v1 = v[1]; s->v2 = v[2]; s->v3 = v[3]; s->v4 = v[4];
    s->d += (uint32_t)offset * 362437u;
}

/* curand_normal (Box-Muller with one cached value), used by the reference's
 * run_daq_many (daq.cu:131).  cuRAND keeps the cache in the state
 * (boxmuller_flag / boxmuller_extra, zeroed by curand_init); here it is a
 * separate 2-word record per slot {flag, extra bits}.  Box-Muller as cuRAND
 * states it: u = x*2^-32 + 2^-33, v = y*(2pi*2^-32) + pi*2^-32,
 * s = sqrt(-2 log u), return s*sin(v), cache s*cos(v).  "Parity unpinned"
 * like the seed salts (no cuRAND in this image). */
CHR_FN float chr_normal(chr_xorwow *s, uint32_t *flag, uint32_t *extra) {
    if (*flag != 1u) {
        const uint32_t x = chr_xorwow_next(s);
        const uint32_t y = chr_xorwow_next(s);
        const float u = (float)x * 2.3283064365386963e-10f + 1.1641532182693481e-10f;
        const float v = (float)y * 1.4629180792671596e-09f + 7.3145903963357980e-10f;
        const float r = chr_sqrtf(-2.0f * chr_logf(u));
        float sv, cv;
        chr_sincosf(v, &sv, &cv);
        *extra = chr_f2u(cv * r);
        *flag = 1u;
        return sv * r;
    }
    *flag = 0u;
    return chr_u2f(*extra);
}

#endif /* CHROMA_RNG_H */
