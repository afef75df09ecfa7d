// bvh_build.cpp -- host-side recursive-grid BVH builder (C ABI chr_bvh_build_grid).
//
// Replaces the reference's GPU-assisted builder: make_recursive_grid_bvh
// (chroma/bvh/grid.py:11-95) with create_leaf_nodes / make_leaves
// (chroma/gpu/bvh.py:18-81, chroma/cuda/bvh.cu:148-203), merge_nodes_detailed /
// make_parents_detailed (gpu/bvh.py:84-112, bvh.cu:269-308), concatenate_layers /
// copy_and_offset (gpu/bvh.py:239-267, bvh.cu:364-384) and collapse_chains /
// collapse_child (gpu/bvh.py:114-130, bvh.cu:530-543).  The reference needs a
// CUDA GPU just to build; the work is a few integer passes, so it runs on the
// host here (OpenMP), and no GPU is needed for config C1.
//
// Node format (bvh/bvh.py:106-195): uint4 {x,y,z: hi16<<16 | lo16 quantised
// bounds, w: nchild<<28 | child}; leaves have nchild == 0 and child = triangle.
//
// Determinism: leaves are ordered by a STABLE radix sort of their Morton codes
// (the reference's numpy quicksort argsort is unstable, so its order among
// equal codes is implementation-defined); quantisation uses IEEE division
// (the reference's --use_fast_math division is approximate).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/chroma_amd.h"
#include "common.h"

namespace {

constexpr uint32_t CHILD_BITS = 28;
constexpr uint32_t MAX_CHILD = (1u << (32 - CHILD_BITS)) - 1;  // 15

struct U4 { uint32_t x, y, z, w; };

inline uint64_t spread3_16(uint32_t v) {
    uint64_t x = v & 0xFFFFu;
    x = (x | (x << 16)) & 0x00000000FF0000FFull;
    x = (x | (x << 8)) & 0x000000F00F00F00Full;
    x = (x | (x << 4)) & 0x00000C30C30C30C3ull;
    x = (x | (x << 2)) & 0x0000249249249249ull;
    return x;
}

inline uint32_t quantize(float v, float origin, float scale) {
    return (uint32_t)((v - origin) / scale);  // truncate (bvh.cu:65-69)
}

// stable LSD radix sort of 48-bit keys, returns permutation
void radix_argsort48(const std::vector<uint64_t> &keys, std::vector<uint32_t> &perm) {
    const size_t n = keys.size();
    std::vector<uint32_t> tmp(n);
    perm.resize(n);
    for (size_t i = 0; i < n; ++i) perm[i] = (uint32_t)i;
    std::vector<size_t> count(1u << 16);
    for (int pass = 0; pass < 3; ++pass) {
        const int shift = 16 * pass;
        std::fill(count.begin(), count.end(), 0);
        for (size_t i = 0; i < n; ++i) count[(keys[perm[i]] >> shift) & 0xFFFFu]++;
        size_t sum = 0;
        for (auto &c : count) { size_t t = c; c = sum; sum += t; }
        for (size_t i = 0; i < n; ++i) tmp[count[(keys[perm[i]] >> shift) & 0xFFFFu]++] = perm[i];
        perm.swap(tmp);
    }
}

inline U4 box_union(const U4 *c, uint32_t n) {
    uint32_t lx = c[0].x & 0xFFFF, ly = c[0].y & 0xFFFF, lz = c[0].z & 0xFFFF;
    uint32_t hx = c[0].x >> 16, hy = c[0].y >> 16, hz = c[0].z >> 16;
    for (uint32_t i = 1; i < n; ++i) {
        lx = std::min(lx, c[i].x & 0xFFFFu); ly = std::min(ly, c[i].y & 0xFFFFu); lz = std::min(lz, c[i].z & 0xFFFFu);
        hx = std::max(hx, c[i].x >> 16); hy = std::max(hy, c[i].y >> 16); hz = std::max(hz, c[i].z >> 16);
    }
    return U4{hx << 16 | lx, hy << 16 | ly, hz << 16 | lz, 0};
}

}  // namespace

struct chr_bvh_result {
    std::vector<U4> nodes;
    std::vector<uint32_t> layer_offsets;
    float world_origin[3];
    float world_scale;
};

extern "C" int chr_bvh_build_grid(const float *h_vertices, uint32_t nvertices, const uint32_t *h_triangles,
                                  uint32_t ntriangles, int32_t target_degree, chr_bvh_result **out) {
    if (!h_vertices || !h_triangles || !out || nvertices == 0 || ntriangles == 0 || target_degree < 1)
        return chr::fail(CHR_ERR_INVALID, "chr_bvh_build_grid: invalid arguments");
    if (ntriangles >= (1u << CHILD_BITS))
        return chr::fail(CHR_ERR_INVALID, "chr_bvh_build_grid: more than 2^28 triangles");
    try {
        auto *res = new chr_bvh_result();
        // world coordinates (gpu/bvh.py:43-48): origin = min vertex, scale = max extent / (2^16-2)
        float lo[3], hi[3];
        for (int a = 0; a < 3; ++a) lo[a] = hi[a] = h_vertices[a];
        for (uint32_t v = 1; v < nvertices; ++v)
            for (int a = 0; a < 3; ++a) {
                float x = h_vertices[3 * (size_t)v + a];
                if (x < lo[a]) lo[a] = x;
                if (x > hi[a]) hi[a] = x;
            }
        float ext = std::max(std::max(hi[0] - lo[0], hi[1] - lo[1]), hi[2] - lo[2]);
        const float scale = ext / 65534.0f;
        const float ox = lo[0], oy = lo[1], oz = lo[2];
        for (int a = 0; a < 3; ++a) res->world_origin[a] = lo[a];
        res->world_scale = scale;

        // leaves + Morton codes (bvh.cu:148-203)
        const size_t n = ntriangles;
        std::vector<U4> leaves(n);
        std::vector<uint64_t> morton(n);
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static)
        for (int64_t t = 0; t < (int64_t)n; ++t) {
            const uint32_t *tri = h_triangles + 3 * t;
            const float *p0 = h_vertices + 3 * (size_t)tri[0];
            const float *p1 = h_vertices + 3 * (size_t)tri[1];
            const float *p2 = h_vertices + 3 * (size_t)tri[2];
            float l[3], u[3], c[3];
            for (int a = 0; a < 3; ++a) {
                l[a] = std::fmin(std::fmin(p0[a], p1[a]), p2[a]);
                u[a] = std::fmax(std::fmax(p0[a], p1[a]), p2[a]);
                c[a] = ((p0[a] + p1[a]) + p2[a]) / 3.0f;
            }
            const float o[3] = {ox, oy, oz};
            uint32_t ql[3], qu[3], qc[3];
            for (int a = 0; a < 3; ++a) {
                ql[a] = quantize(l[a], o[a], scale);
                if (ql[a] > 0) ql[a]--;
                qu[a] = quantize(u[a], o[a], scale) + 1;
                qc[a] = quantize(c[a], o[a], scale);
            }
            morton[t] = spread3_16(qc[0]) | (spread3_16(qc[1]) << 1) | (spread3_16(qc[2]) << 2);
            leaves[t] = U4{ql[0] | (qu[0] << 16), ql[1] | (qu[1] << 16), ql[2] | (qu[2] << 16), (uint32_t)t};
        }

        // Morton order (grid.py:25-28)
        std::vector<uint32_t> perm;
        radix_argsort48(morton, perm);
        std::vector<std::vector<U4>> layers;  // leaf layer first, root last during the build
        {
            std::vector<U4> sorted(n);
            std::vector<uint64_t> sm(n);
            for (size_t i = 0; i < n; ++i) { sorted[i] = leaves[perm[i]]; sm[i] = morton[perm[i]]; }
            leaves.swap(sorted);
            morton.swap(sm);
        }
        layers.push_back(std::move(leaves));

        // parent layers (grid.py:30-91)
        std::vector<uint32_t> first_child, nchild;
        std::vector<uint64_t> parent_morton;
        while (layers.back().size() > 1) {
            const std::vector<U4> &top = layers.back();
            const size_t nnodes = top.size();
            auto count_unique = [&]() {
                size_t u = 1;
                for (size_t i = 1; i < morton.size(); ++i) u += (morton[i] != morton[i - 1]);
                return u;
            };
            size_t nunique = count_unique();
            while ((double)nnodes / (double)nunique < (double)target_degree && nunique > 1) {
                for (auto &m : morton) m >>= 1;
                nunique = count_unique();
            }
            // groups of equal shifted code; groups larger than 15 are cut every 15 children
            first_child.clear(); parent_morton.clear();
            size_t g0 = 0;
            for (size_t i = 1; i <= nnodes; ++i) {
                if (i == nnodes || morton[i] != morton[g0]) {
                    for (size_t f = g0; f < i; f += MAX_CHILD) {
                        first_child.push_back((uint32_t)f);
                        parent_morton.push_back(morton[g0]);
                    }
                    g0 = i;
                }
            }
            const size_t np = first_child.size();
            nchild.resize(np);
            for (size_t p = 0; p < np; ++p)
                nchild[p] = (uint32_t)((p + 1 < np ? first_child[p + 1] : nnodes) - first_child[p]);
            std::vector<U4> parents(np);
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static)
            for (int64_t p = 0; p < (int64_t)np; ++p) {
                U4 b = box_union(&top[first_child[p]], nchild[p]);
                b.w = (nchild[p] << CHILD_BITS) | first_child[p];
                parents[p] = b;
            }
            layers.push_back(std::move(parents));
            morton.swap(parent_morton);
        }

        // concatenate root-first with child offsets (gpu/bvh.py:239-267)
        const size_t nlayers = layers.size();
        std::vector<size_t> bounds(nlayers + 1, 0);
        for (size_t l = 0; l < nlayers; ++l) bounds[l + 1] = bounds[l] + layers[nlayers - 1 - l].size();
        res->nodes.resize(bounds[nlayers]);
        for (size_t l = 0; l < nlayers; ++l) {
            const std::vector<U4> &src = layers[nlayers - 1 - l];
            const uint32_t off = (l + 1 == nlayers) ? 0u : (uint32_t)bounds[l + 1];
            U4 *dst = res->nodes.data() + bounds[l];
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static)
            for (int64_t i = 0; i < (int64_t)src.size(); ++i) {
                U4 v = src[i];
                const uint32_t nc = v.w >> CHILD_BITS, child = v.w & ~(0xFFFFu << CHILD_BITS);
                v.w = (nc << CHILD_BITS) | (child + off);
                dst[i] = v;
            }
            res->layer_offsets.push_back((uint32_t)bounds[l]);
        }
        layers.clear();
        // collapse single-child chains, deepest internal layer first (gpu/bvh.py:114-130)
        for (size_t l = nlayers - 1; l-- > 0;) {
            U4 *nodes = res->nodes.data();
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static)
            for (int64_t i = (int64_t)bounds[l]; i < (int64_t)bounds[l + 1]; ++i) {
                const U4 v = nodes[i];
                if ((v.w >> CHILD_BITS) == 1) nodes[i] = nodes[v.w & ~(0xFFFFu << CHILD_BITS)];
            }
        }
        *out = res;
        return CHR_OK;
    } catch (const std::bad_alloc &) {
        return chr::fail(CHR_ERR_NOMEM, "chr_bvh_build_grid: out of host memory");
    }
}

extern "C" int chr_bvh_result_info(const chr_bvh_result *r, uint32_t *nnodes, uint32_t *nlayers,
                                   float *world_origin, float *world_scale) {
    if (!r) return chr::fail(CHR_ERR_INVALID, "chr_bvh_result_info: null handle");
    if (nnodes) *nnodes = (uint32_t)r->nodes.size();
    if (nlayers) *nlayers = (uint32_t)r->layer_offsets.size();
    if (world_origin) for (int a = 0; a < 3; ++a) world_origin[a] = r->world_origin[a];
    if (world_scale) *world_scale = r->world_scale;
    return CHR_OK;
}

extern "C" int chr_bvh_result_copy(const chr_bvh_result *r, uint32_t *h_nodes, uint32_t *h_layer_offsets) {
    if (!r) return chr::fail(CHR_ERR_INVALID, "chr_bvh_result_copy: null handle");
    if (h_nodes) std::memcpy(h_nodes, r->nodes.data(), r->nodes.size() * sizeof(U4));
    if (h_layer_offsets)
        std::memcpy(h_layer_offsets, r->layer_offsets.data(), r->layer_offsets.size() * sizeof(uint32_t));
    return CHR_OK;
}

extern "C" int chr_bvh_result_free(chr_bvh_result *r) {
    delete r;
    return CHR_OK;
}
