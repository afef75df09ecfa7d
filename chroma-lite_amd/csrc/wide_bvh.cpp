// wide_bvh.cpp -- the gfx950 traversal layout: an 8-wide, SAH-built BVH with
// 8-bit parent-relative child boxes (96-byte nodes), built on the host from
// the reference BVH's own leaf boxes.
//
// Why it exists.  The reference BVH (chroma/bvh/grid.py: Morton-grid groups of
// up to 15 children, one triangle per leaf) makes every ray test ~140-180
// 16-byte nodes in ~30 dependent groups.  A surface-area-heuristic 8-wide tree
// over the SAME leaf boxes tests far fewer nodes, each one 96-byte record.
//
// Why results do not change.  The nearest hit the reference reports is
//   argmin over triangles it TESTS of (distance, position in its DFS order)
// (strict '<', mesh.h:95).  Here:
//   * every triangle's box is the reference leaf box decoded exactly as the
//     reference decodes it (world_origin + q * world_scale, fmaf), and every
//     wide child box contains its triangles' boxes after the kernel's own float
//     decode (checked below), so a ray that passes the reference's slab test on a
//     leaf passes all of ours (the slab test is monotone in the box bounds);
//   * pruning uses the same strict '>' against a running best that is never
//     below the final answer, so the triangles we test include the ones the
//     reference tests;
//   * ties are broken by the reference DFS rank of each triangle (computed
//     here from the reference node array: leaves of a group in index order,
//     then the group's inner children's subtrees in reverse index order).
// Only triangles reachable in the reference BVH are included.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/chroma_amd.h"
#include "common.h"
#include "wide_bvh.h"

namespace chr {
namespace {

constexpr int LEAF_MAX = 4;     // largest leaf the layout holds (kind byte 1..4, 2-bit count in the walk's leaf queue)
// Leaves of at most 3 triangles by default: on the 29k detector trace 14.35 -> 14.10 ms
// per step, 488.4 -> 492.0 M/s, photons identical (profiles/r04/bvh5, two rounds); the
// tail's lone walk is ~2% longer (more nodes per walk) but the trace gain is larger.
constexpr int LEAF_DEFAULT = 3;
// CHR_WIDE_LEAF_MAX=1..4 (build-time A/B of the leaf size; default LEAF_DEFAULT)
inline uint32_t leaf_max_env() {
    const char *e = std::getenv("CHR_WIDE_LEAF_MAX");
    const int v = e ? std::atoi(e) : LEAF_DEFAULT;
    return (uint32_t)std::min(LEAF_MAX, std::max(1, v));
}
// SAH bins per axis.  An exact SAH sweep over every split position of ranges of up
// to 64 triangles found no better tree on these meshes (r04 bvh5: trace 14.35 vs
// 14.41 ms per step, removed).
constexpr int NBINS = 32;

struct Box {
    float lo[3], hi[3];
    void empty() { for (int a = 0; a < 3; ++a) { lo[a] = INFINITY; hi[a] = -INFINITY; } }
    void grow(const Box &b) {
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], b.lo[a]); hi[a] = std::max(hi[a], b.hi[a]); }
    }
    void grow(const float *p) {
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], p[a]); hi[a] = std::max(hi[a], p[a]); }
    }
    double area() const {
        double d[3];
        for (int a = 0; a < 3; ++a) d[a] = std::max(0.0, (double)hi[a] - (double)lo[a]);
        return 2.0 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
};

struct Cluster {
    uint32_t begin, end;
    Box box;
    uint32_t count() const { return end - begin; }
};

struct Builder {
    uint32_t leaf_max;
    const std::vector<Box> &tri_box;
    const std::vector<float> &centroid;   // 3 per triangle
    std::vector<uint32_t> &idx;

    Box range_box(uint32_t b, uint32_t e, bool par) const {
        Box r;
        r.empty();
        if (!par) {
            for (uint32_t i = b; i < e; ++i) r.grow(tri_box[idx[i]]);
            return r;
        }
#pragma omp parallel num_threads(chr::host_threads())
        {
            Box l;
            l.empty();
#pragma omp for schedule(static) nowait
            for (int64_t i = b; i < (int64_t)e; ++i) l.grow(tri_box[idx[i]]);
#pragma omp critical
            r.grow(l);
        }
        return r;
    }

    // binned SAH split of [b,e); returns split point (b < m < e)
    uint32_t split(uint32_t b, uint32_t e, bool par) {
        Box cb;
        cb.empty();
        for (uint32_t i = b; i < e; ++i) cb.grow(&centroid[3 * (size_t)idx[i]]);   // cheap relative to binning
        int best_axis = -1, best_bin = -1;
        double best_cost = INFINITY;
        for (int a = 0; a < 3; ++a) {
            const double ext = (double)cb.hi[a] - (double)cb.lo[a];
            if (!(ext > 0.0)) continue;
            const double k = NBINS / ext * (1.0 - 1e-9);
            Box bins[NBINS];
            uint32_t cnt[NBINS];
            for (int j = 0; j < NBINS; ++j) { bins[j].empty(); cnt[j] = 0; }
            const float lo = cb.lo[a];
            auto bin_of = [&](uint32_t t) {
                int j = (int)(((double)centroid[3 * (size_t)t + a] - lo) * k);
                return std::min(NBINS - 1, std::max(0, j));
            };
            if (par) {
#pragma omp parallel num_threads(chr::host_threads())
                {
                    Box lb[NBINS];
                    uint32_t lc[NBINS];
                    for (int j = 0; j < NBINS; ++j) { lb[j].empty(); lc[j] = 0; }
#pragma omp for schedule(static) nowait
                    for (int64_t i = b; i < (int64_t)e; ++i) {
                        const uint32_t t = idx[i];
                        const int j = bin_of(t);
                        lb[j].grow(tri_box[t]);
                        lc[j]++;
                    }
#pragma omp critical
                    for (int j = 0; j < NBINS; ++j) { bins[j].grow(lb[j]); cnt[j] += lc[j]; }
                }
            } else {
                for (uint32_t i = b; i < e; ++i) {
                    const uint32_t t = idx[i];
                    const int j = bin_of(t);
                    bins[j].grow(tri_box[t]);
                    cnt[j]++;
                }
            }
            double right_area[NBINS];
            uint32_t right_cnt[NBINS];
            Box acc;
            acc.empty();
            uint32_t c = 0;
            for (int j = NBINS - 1; j > 0; --j) {
                acc.grow(bins[j]);
                c += cnt[j];
                right_area[j] = acc.area();
                right_cnt[j] = c;
            }
            acc.empty();
            c = 0;
            for (int j = 0; j < NBINS - 1; ++j) {
                acc.grow(bins[j]);
                c += cnt[j];
                if (c == 0 || right_cnt[j + 1] == 0) continue;
                const double cost = acc.area() * c + right_area[j + 1] * right_cnt[j + 1];
                if (cost < best_cost) { best_cost = cost; best_axis = a; best_bin = j + 1; }
            }
        }
        if (best_axis < 0) return b + (e - b) / 2;   // all centroids coincide: split by count
        const int a = best_axis;
        const double k = NBINS / ((double)cb.hi[a] - (double)cb.lo[a]) * (1.0 - 1e-9);
        const float lo = cb.lo[a];
        auto mid = std::partition(idx.begin() + b, idx.begin() + e, [&](uint32_t t) {
            int j = (int)(((double)centroid[3 * (size_t)t + a] - lo) * k);
            return std::min(NBINS - 1, std::max(0, j)) < best_bin;
        });
        uint32_t m = (uint32_t)(mid - idx.begin());
        if (m == b || m == e) m = b + (e - b) / 2;
        return m;
    }

    // cut [b,e) into <= 8 clusters: repeatedly split the largest-area cluster
    // that holds more than LEAF_MAX triangles; with slots left over, keep
    // splitting multi-triangle leaves (largest area first).  A node costs the
    // same eight slab tests whatever its fill, while leaf triangles are the
    // poorly-converged part of a wave's walk: full nodes, small leaves.
    int clusters(uint32_t b, uint32_t e, bool par, Cluster out[8]) {
        int n = 1;
        out[0] = Cluster{b, e, range_box(b, e, par)};
        while (n < 8) {
            int pick = -1;
            double best = -1.0;
            for (int i = 0; i < n; ++i)
                if (out[i].count() > leaf_max && out[i].box.area() > best) { best = out[i].box.area(); pick = i; }
            if (pick < 0)
                for (int i = 0; i < n; ++i)
                    if (out[i].count() > 1 && out[i].box.area() > best) { best = out[i].box.area(); pick = i; }
            if (pick < 0) break;
            const Cluster c = out[pick];
            const bool p = par && c.count() > (1u << 18);
            const uint32_t m = split(c.begin, c.end, p);
            out[pick] = Cluster{c.begin, m, range_box(c.begin, m, p)};
            out[n++] = Cluster{m, c.end, range_box(m, c.end, p)};
        }
        return n;
    }
};

inline float pow2f(int e) {     // 2^e as float, e in [-126, 127]
    uint32_t u = (uint32_t)(e + 127) << 23;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// quantise one axis of up to 8 child boxes against origin o; returns exponent
// (biased) so that every decoded box contains its child
int quantize_axis(float o, float node_hi, const float *clo, const float *chi, int n, uint8_t *qlo, uint8_t *qhi) {
    const double ext = (double)node_hi - (double)o;
    int e = ext > 0 ? (int)std::ceil(std::log2(ext / 255.0)) : -126;
    e = std::max(-126, std::min(127, e));
    for (;; ++e) {
        const float s = pow2f(e);
        bool ok = true;
        for (int k = 0; k < n && ok; ++k) {
            double fl = std::floor(((double)clo[k] - o) / s), fh = std::ceil(((double)chi[k] - o) / s);
            int l = (int)std::max(0.0, std::min(255.0, fl));
            int h = (int)std::max(0.0, std::min(255.0, fh));
            while (l > 0 && std::fmaf((float)l, s, o) > clo[k]) --l;
            while (h < 255 && std::fmaf((float)h, s, o) < chi[k]) ++h;
            if (std::fmaf((float)l, s, o) > clo[k] || std::fmaf((float)h, s, o) < chi[k]) ok = false;
            qlo[k] = (uint8_t)l;
            qhi[k] = (uint8_t)h;
        }
        if (ok) return e + 127;
        if (e >= 127) return -1;
    }
}

}  // namespace

int build_wide_bvh(const chr_geometry_desc *d, WideBVH &out) {
    const uint32_t ntri = d->ntriangles;
    const float wo[3] = {d->world_origin[0], d->world_origin[1], d->world_origin[2]};
    const float ws = d->world_scale;
    // 1. reference DFS: rank + leaf box per reachable triangle (mesh.h:75-117 order)
    std::vector<uint32_t> rank(ntri, 0xFFFFFFFFu);
    std::vector<Box> tri_box(ntri);
    std::vector<uint32_t> leafq((size_t)ntri * 3);
    out.usable = true;
    {
        auto decode = [&](const uint32_t *n, Box &b) {
            for (int a = 0; a < 3; ++a) {
                b.lo[a] = std::fmaf((float)(n[a] & 0xFFFFu), ws, wo[a]);
                b.hi[a] = std::fmaf((float)(n[a] >> 16), ws, wo[a]);
            }
        };
        const uint32_t *N = d->h_nodes;
        uint32_t next_rank = 0;
        std::vector<uint32_t> stack;
        const uint32_t root_w = N[3];
        if ((root_w >> 28) == 0) {   // a one-triangle mesh: the root is the leaf
            const uint32_t t = root_w & 0x0FFFFFFFu;
            rank[t] = next_rank++;
            decode(N, tri_box[t]);
            std::memcpy(&leafq[3 * (size_t)t], N, 12);
        } else {
            stack.push_back(root_w);
        }
        while (!stack.empty()) {
            const uint32_t w = stack.back();
            stack.pop_back();
            const uint32_t first = w & 0x0FFFFFFFu, end = first + (w >> 28);
            for (uint32_t i = first; i < end; ++i) {
                const uint32_t *n = N + 4 * (size_t)i;
                if ((n[3] >> 28) == 0) {
                    const uint32_t t = n[3] & 0x0FFFFFFFu;
                    if (rank[t] == 0xFFFFFFFFu) {   // first visit defines the tie rank
                        rank[t] = next_rank++;
                        decode(n, tri_box[t]);
                        std::memcpy(&leafq[3 * (size_t)t], n, 12);
                    } else if (std::memcmp(&leafq[3 * (size_t)t], n, 12) != 0) {
                        // a triangle under two different leaf boxes (no builder we
                        // know of makes this): keep the exact-order traversal
                        out.usable = false;
                    }
                } else {
                    stack.push_back(n[3]);
                }
            }
        }
    }
    std::vector<uint32_t> idx;
    idx.reserve(ntri);
    for (uint32_t t = 0; t < ntri; ++t)
        if (rank[t] != 0xFFFFFFFFu) idx.push_back(t);
    const uint32_t nreach = (uint32_t)idx.size();
    std::vector<float> centroid((size_t)ntri * 3);
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static)
    for (int64_t t = 0; t < (int64_t)ntri; ++t)
        for (int a = 0; a < 3; ++a) centroid[3 * t + a] = 0.5f * (tri_box[t].lo[a] + tri_box[t].hi[a]);

    Builder B{leaf_max_env(), tri_box, centroid, idx};
    out.leaf_max = B.leaf_max;
    out.nodes.clear();
    out.tri.clear();
    out.nodes.resize(1);
    out.tri.resize((size_t)nreach * 3);
    if (nreach == 0) {
        std::memset(&out.nodes[0], 0, sizeof(WideNode));
        return CHR_OK;
    }
    struct Task { uint32_t begin, end, node; };
    std::vector<Task> level{Task{0, nreach, 0}};
    uint32_t tri_next = 0;
    while (!level.empty()) {
        const size_t nt = level.size();
        std::vector<Cluster> cl(nt * 8);
        std::vector<int> ncl(nt);
        if (nt < 16) {
            for (size_t i = 0; i < nt; ++i) ncl[i] = B.clusters(level[i].begin, level[i].end, true, &cl[8 * i]);
        } else {
#pragma omp parallel for num_threads(chr::host_threads()) schedule(dynamic, 1)
            for (int64_t i = 0; i < (int64_t)nt; ++i) ncl[i] = B.clusters(level[i].begin, level[i].end, false, &cl[8 * i]);
        }
        // deterministic allocation of child nodes / triangle slots
        std::vector<uint32_t> child_base(nt), tri_base(nt);
        std::vector<Task> next;
        for (size_t i = 0; i < nt; ++i) {
            child_base[i] = (uint32_t)out.nodes.size();
            tri_base[i] = tri_next;
            uint32_t ninner = 0;
            for (int k = 0; k < ncl[i]; ++k) {
                const Cluster &c = cl[8 * i + k];
                if (c.count() > B.leaf_max) {
                    next.push_back(Task{c.begin, c.end, child_base[i] + ninner});
                    ninner++;
                } else {
                    tri_next += c.count();
                }
            }
            out.nodes.resize(out.nodes.size() + ninner);
        }
        int bad = 0;
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static) reduction(+:bad)
        for (int64_t i = 0; i < (int64_t)nt; ++i) {
            WideNode &W = out.nodes[level[i].node];
            std::memset(&W, 0, sizeof(W));
            const int n = ncl[i];
            Box nb;
            nb.empty();
            for (int k = 0; k < n; ++k) nb.grow(cl[8 * i + k].box);
            W.origin[0] = nb.lo[0]; W.origin[1] = nb.lo[1]; W.origin[2] = nb.lo[2];
            W.nchild = (uint8_t)n;
            for (int a = 0; a < 3; ++a) {
                float clo[8], chi[8];
                for (int k = 0; k < n; ++k) { clo[k] = cl[8 * i + k].box.lo[a]; chi[k] = cl[8 * i + k].box.hi[a]; }
                const int e = quantize_axis(nb.lo[a], nb.hi[a], clo, chi, n, W.qlo[a], W.qhi[a]);
                if (e < 0) { bad++; continue; }
                W.exp[a] = (uint8_t)e;
            }
            W.child_base = child_base[i];
            W.tri_base = tri_base[i];
            uint32_t ninner = 0, toff = 0;
            for (int k = 0; k < n; ++k) {
                const Cluster &c = cl[8 * i + k];
                if (c.count() > B.leaf_max) {
                    W.kind[k] = WIDE_INNER;
                    W.off[k] = (uint8_t)ninner++;
                } else {
                    W.kind[k] = (uint8_t)c.count();
                    W.off[k] = (uint8_t)toff;
                    for (uint32_t j = c.begin; j < c.end; ++j) {
                        const uint32_t t = idx[j];
                        const size_t slot = (size_t)W.tri_base + toff++;
                        const uint32_t *ix = d->h_triangles + 3 * (size_t)t;
                        const float *v0 = d->h_vertices + 3 * (size_t)ix[0];
                        const float *v1 = d->h_vertices + 3 * (size_t)ix[1];
                        const float *v2 = d->h_vertices + 3 * (size_t)ix[2];
                        WideTri &R = out.tri[slot];
                        R.v0[0] = v0[0]; R.v0[1] = v0[1]; R.v0[2] = v0[2];
                        for (int a = 0; a < 3; ++a) { R.v1[a] = v1[a]; R.v2[a] = v2[a]; }
                        R.id = t;
                        R.rank = rank[t];
                        std::memcpy(R.leaf, &leafq[3 * (size_t)t], 12);
                        R.code = d->h_material_codes ? d->h_material_codes[t] : 0u;
                        R.pad = 0;
                    }
                }
            }
        }
        if (bad) return chr::fail(CHR_ERR_INVALID, "wide BVH: a node could not be quantised");
        level.swap(next);
        if (!level.empty()) out.max_depth++;
    }
    out.tri.resize(tri_next);
    if (7 * (out.max_depth + 1) + 1 > (uint32_t)WIDE_STACK) out.usable = false;
    return CHR_OK;
}

void wide_compact(const WideBVH &b, std::vector<uint32_t> &rec_id, std::vector<uint32_t> &rec_rank) {
    const int64_t n = (int64_t)b.tri.size();
    rec_id.resize(n);
    rec_rank.resize(n);
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        rec_id[i] = b.tri[i].id;
        rec_rank[i] = b.tri[i].rank;
    }
}

int wide_validate(const chr_geometry_desc *d, const chr_wide_bvh_desc *w, WideCheck &out) {
    if (!w->h_nodes || w->nnodes == 0 || (w->nrec && (!w->h_rec_id || !w->h_rec_rank)))
        return chr::fail(CHR_ERR_INVALID, "wide BVH: missing arrays");
    if (!w->usable) return chr::fail(CHR_ERR_INVALID, "wide BVH: marked unusable (use chr_geometry_create)");
    if (w->nrec > d->ntriangles) return chr::fail(CHR_ERR_INVALID, "wide BVH: %u records > %u triangles", w->nrec, d->ntriangles);
    const WideNode *N = static_cast<const WideNode *>(w->h_nodes);
    const uint32_t nn = w->nnodes, nrec = w->nrec;
    // nodes: children in range and numbered after their parent (the builder allocates a
    // level's children after the level), so one forward pass gives every node's depth
    std::vector<uint16_t> depth(nn, 0);
    uint32_t maxd = 0;
    for (uint32_t i = 0; i < nn; ++i) {
        const WideNode &W = N[i];
        if (W.nchild > 8) return chr::fail(CHR_ERR_INVALID, "wide BVH: node %u has %u children", i, W.nchild);
        for (int k = 0; k < 8; ++k) {
            const uint8_t kind = W.kind[k];
            if (kind == 0) continue;
            if (kind == WIDE_INNER) {
                const uint64_t c = (uint64_t)W.child_base + W.off[k];
                if (c >= nn || c <= i) return chr::fail(CHR_ERR_INVALID, "wide BVH: node %u child %llu out of range", i, (unsigned long long)c);
                const uint32_t dc = depth[i] + 1u;
                if (dc > depth[c]) depth[c] = (uint16_t)std::min<uint32_t>(dc, 0xFFFFu);
                maxd = std::max(maxd, dc);
            } else if (kind <= LEAF_MAX) {
                if ((uint64_t)W.tri_base + W.off[k] + kind > nrec)
                    return chr::fail(CHR_ERR_INVALID, "wide BVH: node %u leaf records out of range", i);
            } else {
                return chr::fail(CHR_ERR_INVALID, "wide BVH: node %u has child kind %u", i, kind);
            }
        }
    }
    if (7 * (maxd + 1) + 1 > (uint32_t)WIDE_STACK)
        return chr::fail(CHR_ERR_INVALID, "wide BVH: depth %u exceeds the walk's stack", maxd);
    if (nn > WIDE_NODE_MASK) return chr::fail(CHR_ERR_INVALID, "wide BVH: %u nodes (walk_up needs < 2^27)", nn);
    // the tree upward: parents (each child has exactly one: the builder's children are
    // disjoint ranges) and every record's leaf node
    out.parent.assign(nn, WIDE_NO_PARENT);
    out.rec_node.assign(nrec, 0u);
    uint32_t *par = out.parent.data(), *rn = out.rec_node.data();
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static)
    for (int64_t i = 0; i < (int64_t)nn; ++i) {
        const WideNode &W = N[i];
        for (int k = 0; k < 8; ++k) {
            const uint8_t kind = W.kind[k];
            if (kind == WIDE_INNER)
                par[W.child_base + W.off[k]] = (uint32_t)i | ((uint32_t)k << 28) | WIDE_ANCESTOR;
            else if (kind != 0)
                for (uint32_t t = 0; t < kind; ++t) rn[W.tri_base + W.off[k] + t] = (uint32_t)i;
        }
    }
    // records: triangle ids in range, ranks a permutation of [0, nrec)
    out.rank_rec.assign(nrec, 0xFFFFFFFFu);
    int bad = 0;
    uint32_t *rr = out.rank_rec.data();
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static) reduction(| : bad)
    for (int64_t i = 0; i < (int64_t)nrec; ++i) {
        const uint32_t r = w->h_rec_rank[i];
        if (r >= nrec || w->h_rec_id[i] >= d->ntriangles) { bad = 1; continue; }
        __atomic_store_n(rr + r, (uint32_t)i, __ATOMIC_RELAXED);
    }
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static) reduction(| : bad)
    for (int64_t r = 0; r < (int64_t)nrec; ++r)
        if (rr[r] == 0xFFFFFFFFu) bad = 1;       // a rank missing: some other rank repeats
    if (bad) return chr::fail(CHR_ERR_INVALID, "wide BVH: record ids out of range or ranks not a permutation");
    // reference leaf words per triangle (a triangle under several leaves has the same
    // words under each in a usable tree, wide_bvh.cpp build step 1)
    const size_t nt = d->ntriangles;
    out.leafq.assign(3 * nt, 0u);
    std::vector<uint8_t> has(nt, 0);
    uint32_t *lq = out.leafq.data();
    uint8_t *hp = has.data();
    const uint32_t *RN = d->h_nodes;
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static)
    for (int64_t i = 0; i < (int64_t)d->nnodes; ++i) {
        const uint32_t *n = RN + 4 * (size_t)i;
        if ((n[3] >> 28) != 0) continue;
        const uint32_t t = n[3] & 0x0FFFFFFFu;
        if (t >= nt) continue;
        for (int a = 0; a < 3; ++a) __atomic_store_n(lq + 3 * (size_t)t + a, n[a], __ATOMIC_RELAXED);
        __atomic_store_n(hp + t, (uint8_t)1, __ATOMIC_RELAXED);
    }
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static) reduction(| : bad)
    for (int64_t i = 0; i < (int64_t)nrec; ++i)
        if (!hp[w->h_rec_id[i]]) bad = 1;
    if (bad) return chr::fail(CHR_ERR_INVALID, "wide BVH: a record's triangle is under no reference leaf");
    return CHR_OK;
}

void wide_fill_records(const chr_geometry_desc *d, const chr_wide_bvh_desc *w, const WideCheck &c, size_t first,
                       size_t n, WideTri *out) {
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static)
    for (int64_t j = 0; j < (int64_t)n; ++j) {
        const size_t i = first + (size_t)j;
        const uint32_t t = w->h_rec_id[i];
        const uint32_t *ix = d->h_triangles + 3 * (size_t)t;
        WideTri &R = out[j];
        for (int a = 0; a < 3; ++a) {
            R.v0[a] = d->h_vertices[3 * (size_t)ix[0] + a];
            R.v1[a] = d->h_vertices[3 * (size_t)ix[1] + a];
            R.v2[a] = d->h_vertices[3 * (size_t)ix[2] + a];
        }
        R.id = t;
        R.rank = w->h_rec_rank[i];
        std::memcpy(R.leaf, &c.leafq[3 * (size_t)t], 12);
        R.code = d->h_material_codes ? d->h_material_codes[t] : 0u;
        R.pad = c.rec_node.empty() ? 0u : c.rec_node[i];
    }
}

void wide_fill_node_slots(const chr_wide_bvh_desc *w, const WideCheck &c, size_t first, size_t n, uint8_t *out) {
    const WideNode *N = static_cast<const WideNode *>(w->h_nodes);
    const uint32_t *par = c.parent.data();
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static)
    for (int64_t j = 0; j < (int64_t)n; ++j) {
        uint8_t *slot = out + 128 * (size_t)j;
        std::memcpy(slot, N + first + (size_t)j, sizeof(WideNode));
        uint32_t chain[8];
        uint32_t a = (uint32_t)(first + (size_t)j);
        for (int m = 0; m < 8; ++m) {
            const uint32_t p = a == WIDE_NO_PARENT || c.parent.empty() ? WIDE_NO_PARENT : par[a];
            chain[m] = p;
            a = p == WIDE_NO_PARENT ? WIDE_NO_PARENT : (p & WIDE_NODE_MASK);
        }
        if (a != WIDE_NO_PARENT && !c.parent.empty() && par[a] != WIDE_NO_PARENT) chain[7] |= WIDE_CHAIN_MORE;
        std::memcpy(slot + sizeof(WideNode), chain, sizeof(chain));
    }
}

}  // namespace chr

struct chr_wide_result {
    chr::WideBVH b;
};

extern "C" int chr_wide_bvh_build(const chr_geometry_desc *d, chr_wide_result **out) {
    if (!d || !out || !d->h_nodes || !d->h_vertices || !d->h_triangles || d->nnodes == 0)
        return chr::fail(CHR_ERR_INVALID, "chr_wide_bvh_build: null argument or empty BVH");
    chr_wide_result *r = new (std::nothrow) chr_wide_result();
    if (!r) return chr::fail(CHR_ERR_NOMEM, "chr_wide_bvh_build: host allocation failed");
    const int rc = chr::build_wide_bvh(d, r->b);
    if (rc) { delete r; return rc; }
    *out = r;
    return CHR_OK;
}

extern "C" int chr_wide_bvh_info(const chr_wide_result *r, uint32_t *nnodes, uint32_t *ntri, uint32_t *max_depth,
                                 int32_t *usable) {
    if (!r) return chr::fail(CHR_ERR_INVALID, "chr_wide_bvh_info: null handle");
    if (nnodes) *nnodes = (uint32_t)r->b.nodes.size();
    if (ntri) *ntri = (uint32_t)r->b.tri.size();
    if (max_depth) *max_depth = r->b.max_depth;
    if (usable) *usable = r->b.usable ? 1 : 0;
    return CHR_OK;
}

extern "C" int chr_wide_bvh_copy(const chr_wide_result *r, void *h_nodes, void *h_tri) {
    if (!r) return chr::fail(CHR_ERR_INVALID, "chr_wide_bvh_copy: null handle");
    if (h_nodes) std::memcpy(h_nodes, r->b.nodes.data(), r->b.nodes.size() * sizeof(chr::WideNode));
    if (h_tri) std::memcpy(h_tri, r->b.tri.data(), r->b.tri.size() * sizeof(chr::WideTri));
    return CHR_OK;
}

extern "C" int chr_wide_bvh_free(chr_wide_result *r) {
    delete r;
    return CHR_OK;
}

extern "C" int chr_wide_bvh_describe(const chr_wide_result *r, chr_wide_bvh_desc *out) {
    if (!r || !out) return chr::fail(CHR_ERR_INVALID, "chr_wide_bvh_describe: null argument");
    std::memset(out, 0, sizeof(*out));
    out->nnodes = (uint32_t)r->b.nodes.size();
    out->nrec = (uint32_t)r->b.tri.size();
    out->max_depth = r->b.max_depth;
    out->usable = r->b.usable ? 1 : 0;
    out->leaf_max = r->b.leaf_max;
    return CHR_OK;
}

extern "C" int chr_wide_bvh_export(const chr_wide_result *r, void *h_nodes, uint32_t *h_rec_id,
                                   uint32_t *h_rec_rank) {
    if (!r) return chr::fail(CHR_ERR_INVALID, "chr_wide_bvh_export: null handle");
    if (h_nodes) std::memcpy(h_nodes, r->b.nodes.data(), r->b.nodes.size() * sizeof(chr::WideNode));
    if (h_rec_id || h_rec_rank) {
        const int64_t n = (int64_t)r->b.tri.size();
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            if (h_rec_id) h_rec_id[i] = r->b.tri[i].id;
            if (h_rec_rank) h_rec_rank[i] = r->b.tri[i].rank;
        }
    }
    return CHR_OK;
}

extern "C" int chr_wide_bvh_key(char *out, uint32_t n) {
    if (!out || n == 0) return chr::fail(CHR_ERR_INVALID, "chr_wide_bvh_key: no buffer");
    // bump the format number whenever the builder's output for the same inputs changes
    const int len = std::snprintf(out, n, "w%d-l%u", chr::WIDE_FORMAT, chr::leaf_max_env());
    if (len < 0 || (uint32_t)len >= n) return chr::fail(CHR_ERR_INVALID, "chr_wide_bvh_key: buffer too small");
    return CHR_OK;
}

extern "C" int chr_wide_bvh_records(const chr_geometry_desc *d, const chr_wide_bvh_desc *w, uint32_t first, uint32_t n,
                                    void *h_tri) {
    if (!d || !w || (n && !h_tri)) return chr::fail(CHR_ERR_INVALID, "chr_wide_bvh_records: null argument");
    if ((uint64_t)first + n > w->nrec) return chr::fail(CHR_ERR_INVALID, "chr_wide_bvh_records: range past the records");
    try {
        chr::WideCheck c;
        if (int rc = chr::wide_validate(d, w, c)) return rc;
        chr::wide_fill_records(d, w, c, first, n, static_cast<chr::WideTri *>(h_tri));
    } catch (const std::bad_alloc &) {
        return chr::fail(CHR_ERR_NOMEM, "chr_wide_bvh_records: out of host memory");
    }
    return CHR_OK;
}
