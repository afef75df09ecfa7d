// unique.cpp -- chr_unique_vertices: the vertex merge of Geometry.flatten
// (np.unique over (x, y, z) rows with return_inverse, chroma/geometry.py:71-81)
// as a parallel sort on the host.  numpy sorts the rows as structured values
// (field by field, float comparison: -0.0 == +0.0) and keeps the first row of
// each equal run.  When every equal run is bit-identical the result is the
// same whichever duplicate a sort puts first; inputs with a NaN, or with a run
// mixing +0.0 and -0.0, are refused (the caller keeps numpy's answer).
#include <parallel/algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/chroma_amd.h"
#include "common.h"

namespace {

// order-preserving map of a float (no NaN) to an unsigned key; -0.0 maps to
// +0.0's key (they compare equal, as in numpy's structured comparison)
inline uint32_t fkey(uint32_t u) {
    if (u == 0x80000000u) u = 0u;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

struct Row {
    uint64_t xy;     // key(x) << 32 | key(y)
    uint32_t z;      // key(z)
    uint32_t idx;    // input row (< 2^32)
    bool operator<(const Row &o) const { return xy != o.xy ? xy < o.xy : (z != o.z ? z < o.z : idx < o.idx); }
    bool same(const Row &o) const { return xy == o.xy && z == o.z; }
};

}  // namespace

extern "C" int chr_unique_vertices(const float *v, uint64_t n, float *out, uint64_t *nunique, int64_t *inverse) {
    if (!nunique || (n && (!v || !out || !inverse))) return chr::fail(CHR_ERR_INVALID, "chr_unique_vertices: null argument");
    if (n >= (1ull << 32)) return chr::fail(CHR_ERR_INVALID, "chr_unique_vertices: more than 2^32-1 rows");
    *nunique = 0;
    if (n == 0) return CHR_OK;
    const uint32_t *u = reinterpret_cast<const uint32_t *>(v);
    std::vector<Row> rows(n);
    int bad = 0;
#pragma omp parallel for num_threads(chr::host_threads()) reduction(| : bad) schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        uint32_t k[3];
        for (int c = 0; c < 3; ++c) {
            const uint32_t b = u[3 * i + c];
            if ((b & 0x7F800000u) == 0x7F800000u && (b & 0x007FFFFFu)) bad = 1;   // NaN
            k[c] = fkey(b);
        }
        rows[i] = Row{((uint64_t)k[0] << 32) | k[1], k[2], (uint32_t)i};
    }
    if (bad) return chr::fail(CHR_ERR_INVALID, "chr_unique_vertices: NaN present");
    __gnu_parallel::sort(rows.begin(), rows.end(), __gnu_parallel::default_parallel_tag(chr::host_threads()));
    // group starts -> unique row numbers (prefix count, in parallel blocks)
    const int64_t N = (int64_t)n;
    std::vector<uint8_t> start(n);
    int mixed = 0;
#pragma omp parallel for num_threads(chr::host_threads()) reduction(| : mixed) schedule(static)
    for (int64_t j = 0; j < N; ++j) {
        start[j] = (j == 0 || !rows[j].same(rows[j - 1])) ? 1 : 0;
        // an equal run holding both zeros of a coordinate: which row numpy keeps
        // depends on its (unstable) sort -- not decidable here
        if (!start[j] && std::memcmp(v + 3 * (size_t)rows[j].idx, v + 3 * (size_t)rows[j - 1].idx, 12) != 0) mixed = 1;
    }
    if (mixed) return chr::fail(CHR_ERR_INVALID, "chr_unique_vertices: +0.0 and -0.0 in one set of equal rows");
    std::vector<int64_t> gid(n);
    int64_t g = -1;
    for (int64_t j = 0; j < N; ++j) {   // sequential scan: ~n byte reads
        g += start[j];
        gid[j] = g;
    }
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static)
    for (int64_t j = 0; j < N; ++j) {
        const uint32_t i = rows[j].idx;
        inverse[i] = gid[j];
        if (start[j]) std::memcpy(out + 3 * gid[j], v + 3 * (size_t)i, 12);
    }
    *nunique = (uint64_t)(g + 1);
    return CHR_OK;
}
