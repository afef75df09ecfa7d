// propagate.hip -- gfx950 photon propagation kernels + their C ABI.
//
// Hot path: the `propagate` kernel of the reference (chroma/cuda/propagate.cu:
// 254-366) with everything it inlines from photon.h (fill_state, propagate_to_
// boundary, propagate_at_surface, propagate_at_boundary), mesh.h
// (intersect_mesh) and intersect.h.  Restructured for CDNA4:
//   * one work-item per queue slot, 256-thread workgroups (4 waves of 64);
//   * the BVH walk keeps the reference's DFS order and 1000-entry stack
//     semantics, but the top STACK_LDS entries live in LDS (lane-strided, bank
//     conflict free) and only deeper entries spill to private scratch;
//   * triangles are fetched as one 48-byte de-indexed record (device_geometry.h);
//   * the RNG state (cuRAND-compatible XORWOW) sits in VGPRs for the whole
//     launch; slot states are stored SoA so the six words load/store coalesced;
//   * survivors are compacted with a wave64 ballot mask per 64 slots, an
//     exclusive scan of the mask popcounts and an order-preserving scatter
//     (the reference's warp-atomic enqueue is nondeterministic);
//   * all transcendental math is include/chroma_fmath.h, bit-identical to the
//     CPU oracle.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <type_traits>
#include <vector>

#include "../../include/chroma_amd.h"
#include "../../include/chroma_fmath.h"
#include "../../include/chroma_rng.h"
#include "common.h"
#include "device_geometry.h"
#include "device_math.h"
#include "sampling.h"
#include "wide_bvh.h"

namespace chr {

constexpr int BLOCK = 256;
constexpr int STACK_SIZE = 1000;   // mesh.h:10
constexpr int STACK_LDS = 24;      // entries kept in LDS per work-item
constexpr uint32_t DEAD_MASK = CHR_NO_HIT | CHR_BULK_ABSORB | CHR_SURFACE_DETECT | CHR_SURFACE_ABSORB | CHR_NAN_ABORT;
constexpr float WEIGHT_LOWER_THRESHOLD = 0.0001f;
constexpr float SPEED_OF_LIGHT = 299.792458f;
// float thresholds equivalent to the reference's float-vs-double compares
// (intersect.h:259-267): (double)u < -1e-6, (double)u > 1+1e-6, (double)t > 1e-6
constexpr float T_NEG_EPS = -9.99999997e-07f;
constexpr float T_ONE_EPS = 1.00000095367431640625f;
constexpr float T_POS_EPS = 9.99999997e-07f;

enum { BREAK = 0, CONTINUE = 1, PASS = 2 };

struct Photon {
    V3 pos, dir, pol;
    float wavelength, time, weight;
    uint32_t history;   // holds a 16-bit value (photon.h:29)
    int last_hit;
};

struct State {
    V3 normal;
    float n1, n2, absorption_length, scattering_length, distance;
    int material1, surface_index;
    bool inside_to_outside;   // photon.h:38 (the hybrid renderer reads it)
};

#define CHR_LDS __attribute__((address_space(3)))
#ifndef CHR_COLD
#define CHR_COLD __forceinline__
#endif
// The LDS column pointer travels as a plain value (never inside an object that
// also holds the scratch spill array: such an object lives in scratch and its
// LDS pointer degrades to flat loads/stores).
struct Stack {
    CHR_LDS uint32_t *lds;   // this work-item's column: entry i at lds[i * BLOCK]
};

__device__ __forceinline__ void stack_put(const Stack &s, uint32_t *spill, int i, uint32_t v) {
    if (i < STACK_LDS) s.lds[i * BLOCK] = v;
    else spill[i - STACK_LDS] = v;
}
__device__ __forceinline__ uint32_t stack_get(const Stack &s, const uint32_t *spill, int i) {
    return (i < STACK_LDS) ? s.lds[i * BLOCK] : spill[i - STACK_LDS];
}

// Loads through pointers fetched from the device-resident DevGeom are flat
// (generic) loads unless the address space is stated; flat loads also count in
// lgkmcnt and so serialise against the LDS stack.  gld() = global_load.
#define CHR_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ T gld(const T *p) { return *(const CHR_GLOBAL T *)p; }
typedef uint32_t chr_u32x4 __attribute__((ext_vector_type(4)));
typedef float chr_f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gld(const uint4 *p) {
    const chr_u32x4 v = *(const CHR_GLOBAL chr_u32x4 *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float4 gld(const float4 *p) {
    const chr_f32x4 v = *(const CHR_GLOBAL chr_f32x4 *)p;
    return make_float4(v.x, v.y, v.z, v.w);
}
typedef uint32_t chr_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 gld_lo2(const void *p) {   // the first 8 bytes at p (global_load_dwordx2)
    const chr_u32x2 v = *(const CHR_GLOBAL chr_u32x2 *)p;
    return make_uint2(v.x, v.y);
}

// ---------------------------------------------------------------- geometry.h
// The top of the wide BVH in LDS (north_star: "BVH nodes ... staged through
// LDS").  The builder numbers nodes level by level (wide_bvh.cpp), so nodes
// [0, TOP_NODES) are the root and the two levels below it of the 8-wide tree:
// every walk starts there and re-enters them from its stack.  A workgroup copies
// them once (96 B each: the node without its slot pad); a walk reads node i < n
// from LDS, every other node from global memory.  Same bytes, same results.
constexpr uint32_t TOP_NODES = 73;   // 1 + 8 + 64: 7,008 B
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // (HIP's uint4 has no LDS assignment)
struct TopNodes {
    const CHR_LDS u32x4 *p;          // 6 x 16 B per node
    uint32_t n;                      // nodes held (0: none)
};
template <int TB>
__device__ __forceinline__ TopNodes stage_top(const DevGeom &g, CHR_LDS u32x4 *lds, uint32_t want) {
    const uint32_t n = want < g.nwnodes ? want : g.nwnodes;   // workgroup-uniform
    for (uint32_t i = threadIdx.x; i < 6u * n; i += TB) {
        const uint4 v = gld(g.wnodes + (size_t)g.wstride * (i / 6u) + i % 6u);
        u32x4 w;
        w.x = v.x; w.y = v.y; w.z = v.z; w.w = v.w;
        lds[i] = w;
    }
    __syncthreads();
    return TopNodes{lds, n};
}
__device__ __forceinline__ uint4 u4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ void load_node(const DevGeom &g, const TopNodes &top, uint32_t node, uint4 &h, uint4 &a1,
                                          uint4 &a2, uint4 &a3, uint4 &a4, uint4 &a5) {
    if (node < top.n) {
        const CHR_LDS u32x4 *tp = top.p + 6u * node;
        h = u4(tp[0]); a1 = u4(tp[1]); a2 = u4(tp[2]); a3 = u4(tp[3]); a4 = u4(tp[4]); a5 = u4(tp[5]);
    } else {
        const uint4 *np = g.wnodes + (size_t)g.wstride * node;
        h = gld(np); a1 = gld(np + 1); a2 = gld(np + 2); a3 = gld(np + 3); a4 = gld(np + 4); a5 = gld(np + 5);
    }
}

__device__ __forceinline__ void node_bounds(const DevGeom &g, uint4 n, V3 &lo, V3 &hi) {
    lo = v3(__builtin_fmaf((float)(n.x & 0xFFFFu), g.scale, g.ox), __builtin_fmaf((float)(n.y & 0xFFFFu), g.scale, g.oy),
            __builtin_fmaf((float)(n.z & 0xFFFFu), g.scale, g.oz));
    hi = v3(__builtin_fmaf((float)(n.x >> 16), g.scale, g.ox), __builtin_fmaf((float)(n.y >> 16), g.scale, g.oy),
            __builtin_fmaf((float)(n.z >> 16), g.scale, g.oz));
}

// a table word: from LDS when the tables were copied there (phys_cache), else a global load
__device__ __forceinline__ float tab(const float *p) {
    return __builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void *)p) ? *(const CHR_LDS float *)p
                                                                                         : gld(p);
}
__device__ __forceinline__ float interp_property(const DevGeom &g, float x, const float *fp) {
    const float start = g.wl_start, step = g.wl_step;
    const int n = (int)g.wl_n;
    if (x < start) return tab(fp);
    if (x > __builtin_fmaf((float)(n - 1), step, start)) return tab(fp + n - 1);
    const int jl = (int)((x - start) / step);
    const float base = __builtin_fmaf((float)jl, step, start);
    const float f0 = tab(fp + jl), f1 = tab(fp + jl + 1);
    return f0 + ((x - base) * (f1 - f0)) / step;
}

// ---------------------------------------------------------------- intersect.h / mesh.h
__device__ __forceinline__ bool intersect_box(V3 noid, V3 inv, V3 lo, V3 hi, float &dist) {
    float tmin = 0.0f, tmax = __builtin_inff();
    if (chr_isfinite(inv.x)) {
        const float t0 = __builtin_fmaf(lo.x, inv.x, noid.x), t1 = __builtin_fmaf(hi.x, inv.x, noid.x);
        tmin = fmax_(tmin, fmin_(t0, t1)); tmax = fmin_(tmax, fmax_(t0, t1));
    }
    if (chr_isfinite(inv.y)) {
        const float t0 = __builtin_fmaf(lo.y, inv.y, noid.y), t1 = __builtin_fmaf(hi.y, inv.y, noid.y);
        tmin = fmax_(tmin, fmin_(t0, t1)); tmax = fmin_(tmax, fmax_(t0, t1));
    }
    if (chr_isfinite(inv.z)) {
        const float t0 = __builtin_fmaf(lo.z, inv.z, noid.z), t1 = __builtin_fmaf(hi.z, inv.z, noid.z);
        tmin = fmax_(tmin, fmin_(t0, t1)); tmax = fmin_(tmax, fmax_(t0, t1));
    }
    if (tmin > tmax) return false;
    dist = tmin;
    return true;
}

// Moller-Trumbore on a de-indexed record (v0, e1, e2)
__device__ __forceinline__ bool intersect_triangle(V3 o, V3 d, V3 v0, V3 e1, V3 e2, float &distance) {
    const V3 h = cross(d, e2);
    const float a = dot(e1, h);
    if (a > -1.19209290e-7f && a < 1.19209290e-7f) return false;
    const float f = 1.0f / a;
    const V3 s = o - v0;
    const float u = f * dot(s, h);
    if (u < T_NEG_EPS || u > T_ONE_EPS) return false;
    const V3 q = cross(s, e1);
    const float v = f * dot(d, q);
    if (v < T_NEG_EPS || u + v > T_ONE_EPS) return false;
    const float t = f * dot(e2, q);
    if (t > T_POS_EPS && t < __builtin_inff()) {
        distance = t;
        return true;
    }
    return false;
}

// Moller-Trumbore on a wide-BVH triangle record (wide_bvh.h: v0, v1, v2 in
// r0..r2): the edges v1-v0, v2-v0 are the reference's own float subtractions
// (intersect.h:26-101), so this is intersect_triangle on the same operands.
__device__ __forceinline__ bool intersect_record(V3 o, V3 d, float4 r0, float4 r1, float4 r2, float &distance) {
    const V3 v0 = v3(r0.x, r0.y, r0.z), v1 = v3(r0.w, r1.x, r1.y), v2 = v3(r1.z, r1.w, r2.x);
    return intersect_triangle(o, d, v0, v1 - v0, v2 - v0, distance);
}
// the record index of a wide-BVH triangle record pointer: what the wide walks
// return for a hit (finish_fill<true> reads the triangle id and normal from it)
__device__ __forceinline__ int rec_of(const DevGeom &g, const float4 *r) { return (int)((r - g.wtri) >> 2); }

// mesh.h:45-126 -- nearest triangle != last_hit; reference DFS order.
// The children of a popped group are fetched BATCH at a time (independent
// 16-byte loads in flight together), their slab tests computed up front, and
// then walked strictly in index order with the reference's prune / accept /
// push decisions, so the result (including tie-breaking) is unchanged.
template <int BATCH>
__device__ __forceinline__ int intersect_mesh(const DevGeom &g, V3 o, V3 d, float &min_distance, int last_hit,
                                              Stack st, uint32_t &overflow) {
    uint32_t spill[STACK_SIZE - STACK_LDS];
    int triangle_index = -1;
    min_distance = -1.0f;
    const V3 noid = v3(-o.x / d.x, -o.y / d.y, -o.z / d.z);
    const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const uint4 root = gld(g.nodes);
    {
        V3 lo, hi;
        float bd;
        node_bounds(g, root, lo, hi);
        if (!intersect_box(noid, inv, lo, hi, bd)) return -1;
    }
    stack_put(st, spill, 0, root.w);
    int curr = 0;
    const uint32_t last = (uint32_t)last_hit;
    while (curr >= 0) {
        const uint32_t w = stack_get(st, spill, curr);
        curr--;
        const uint32_t end = (w & 0x0FFFFFFFu) + (w >> 28);
        for (uint32_t i = w & 0x0FFFFFFFu; i < end; i += BATCH) {
            uint4 nd[BATCH];
#pragma unroll
            for (int k = 0; k < BATCH; ++k)
                if (i + k < end) nd[k] = gld(g.nodes + i + k);
            float bd[BATCH];
            bool hit[BATCH];
#pragma unroll
            for (int k = 0; k < BATCH; ++k) {
                V3 lo, hi;
                node_bounds(g, nd[k], lo, hi);
                hit[k] = (i + k < end) && intersect_box(noid, inv, lo, hi, bd[k]);
            }
#pragma unroll
            for (int k = 0; k < BATCH; ++k) {
                if (!hit[k]) continue;
                if (min_distance >= 0.0f && bd[k] > min_distance) continue;
                const uint32_t child = nd[k].w & 0x0FFFFFFFu;
                if ((nd[k].w >> 28) == 0) {
                    if (child != last) {
                        const float4 *r = g.tri + 3 * (size_t)child;
                        const float4 r0 = gld(r), r1 = gld(r + 1), r2 = gld(r + 2);
                        float dist;
                        if (intersect_triangle(o, d, v3(r0.x, r0.y, r0.z), v3(r0.w, r1.x, r1.y), v3(r1.z, r1.w, r2.x),
                                               dist)) {
                            if (triangle_index == -1 || dist < min_distance) {
                                triangle_index = (int)child;
                                min_distance = dist;
                            }
                        }
                    }
                } else {
                    if (curr + 1 >= STACK_SIZE) {
                        overflow++;
                        return triangle_index;
                    }
                    curr++;
                    stack_put(st, spill, curr, nd[k].w);
                }
            }
        }
    }
    return triangle_index;
}

// ---------------------------------------------------------------- wide traversal
// The same nearest-hit query over the 8-wide SAH BVH (wide_bvh.h).  Each
// triangle is still admitted by the reference's own leaf test (slab test of
// its reference leaf box + prune `box distance > best`), then Moller-Trumbore,
// and the winner is the minimum of (distance, reference DFS rank) -- exactly
// the triangle the reference's strict-'<' DFS keeps (wide_bvh.cpp explains
// why the tested set covers the reference's).  Stack: top WIDE_LDS entries
// (node, entry distance) in LDS, the rest in scratch; nearest inner child
// first, the others pushed and culled at pop against the running best.
constexpr int WIDE_LDS = 12;
constexpr int LEAFQ = 16;          // per-lane parked-leaf queue (speculative walk), LDS
// LDS words per work-item: traversal stack (node + entry distance) [+ leaf queue]
constexpr int lds_words(int wide) { return wide >= 2000 ? 2 * WIDE_LDS + LEAFQ : (wide ? 2 * WIDE_LDS : 0); }

// The LDS column pointers are typed (ds_* ops) and the scratch spill array is
// a separate object: an object holding both lives in scratch and its LDS
// pointers degrade to flat ops behind a scratch load (measured r01: the
// scheduled walk runs 1.14x faster this way).
struct WStack {
    CHR_LDS uint32_t *node;   // this work-item's LDS column: entry i at node[i * BLOCK]
    CHR_LDS float *dist;
    uint2 *spill;             // entries >= SL: private array (sstride 1) or a lane-strided HBM column
    uint32_t sstride;         // uint2 between consecutive spill entries of this work-item
    CHR_LDS uint32_t *leafq;  // parked leaves (speculative walk): entry i at leafq[i * BLOCK]
};
// SL: stack entries kept in LDS (the rest spill to scratch)
// TB: the LDS column stride (threads of the workgroup: trace_kernel may run
// wider workgroups than BLOCK, so its per-CU top-of-tree copy is shared by more waves)
template <int SL = WIDE_LDS, int TB = BLOCK>
__device__ __forceinline__ void wpush(WStack &s, int i, uint32_t n, float t) {
    if (i < SL) { s.node[i * TB] = n; s.dist[i * TB] = t; }
    else s.spill[(size_t)(i - SL) * s.sstride] = make_uint2(n, __float_as_uint(t));
}
template <int SL = WIDE_LDS, int TB = BLOCK>
__device__ __forceinline__ void wpop(const WStack &s, int i, uint32_t &n, float &t) {
    if (i < SL) { n = s.node[i * TB]; t = s.dist[i * TB]; }
    else { const uint2 e = s.spill[(size_t)(i - SL) * s.sstride]; n = e.x; t = __uint_as_float(e.y); }
}

__device__ __forceinline__ float byte_f(uint32_t lo4, uint32_t hi4, int k) {   // byte k of (hi4:lo4) as float
    const uint32_t w = k < 4 ? lo4 : hi4;
    return (float)((w >> (8 * (k & 3))) & 0xFFu);
}
__device__ __forceinline__ float exp_scale(uint32_t e) { return __uint_as_float((e & 0xFFu) << 23); }
typedef float F2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ F2 f2(float a, float b) { F2 v; v.x = a; v.y = b; return v; }
__device__ __forceinline__ F2 pk_fma(F2 a, F2 b, F2 c) { return __builtin_elementwise_fma(a, b, c); }

// Per-ray constants of the branch-free slab test used on wide nodes.  For an
// axis with finite 1/d the near/far plane distances are fmaf(x, inv, noid) --
// the reference's own expression (intersect_box, intersect.h:113-157), and
// since fmaf is monotone in x, selecting the near/far bound by the sign of
// inv gives exactly the min/max the reference takes.
// A FLAT axis (1/d not finite: d = +-0 or denormal) is skipped by the
// reference's box test, so its DFS enters every box the ray's projection
// crosses (one such walk took 19 s in round 1; rounds 2-4 split it into 2^18
// sub-walks shared by the grid).  The traversal here instead tests that axis
// as what it is, the ray's constant coordinate o inside [lo, hi]: multiplier
// 2^100 and offset -o * 2^100 (both exact), so fmaf(x, 2^100, -o * 2^100) is
// (x - o) * 2^100 rounded once -- negative, zero or positive exactly as x - o.
// The nearest hit is unchanged: a triangle the ray hits holds a point at the
// ray's coordinate on that axis (up to Moller-Trumbore's 1e-6 barycentric
// tolerance, ~1e-5 mm), and its reference leaf box extends at least one
// quantum (world_scale, ~0.7 mm on the 29k detector) beyond its vertices
// (bvh.cu make_leaves: lower - 1, upper + 1), so every box on the way to it
// holds o on that axis; the traversal only skips boxes that hold no hit.  (The
// one exception: a leaf box at the world minimum (quantised lower bound 0 gets
// no margin) hit by a ray lying within that tolerance outside the world box.)
// The leaf-box acceptance of a candidate (intersect_box_slab) keeps the
// reference's skip of the flat axis (RaySlab::flat).
struct RaySlab {
    float inx, iny, inz;        // multipliers (inv, or 2^100 on a flat axis)
    float onx, ony, onz;        // near offsets (noid, or -o * 2^100)
    float ofx, ofy, ofz;        // far offsets (same)
    bool negx, negy, negz;      // inv < 0: the near plane is the box's hi face
    uint32_t flat;              // bit k: axis k flat (skipped by intersect_box_slab, as the reference does)
};
__device__ __forceinline__ RaySlab make_slab(V3 o, V3 noid, V3 inv) {
    RaySlab r;
    constexpr float BIG = 1.2676506e30f;   // 2^100
    const bool fx = chr_isfinite(inv.x), fy = chr_isfinite(inv.y), fz = chr_isfinite(inv.z);
    r.inx = fx ? inv.x : BIG; r.onx = fx ? noid.x : -(o.x * BIG); r.ofx = r.onx;
    r.iny = fy ? inv.y : BIG; r.ony = fy ? noid.y : -(o.y * BIG); r.ofy = r.ony;
    r.inz = fz ? inv.z : BIG; r.onz = fz ? noid.z : -(o.z * BIG); r.ofz = r.onz;
    r.negx = fx && inv.x < 0.0f; r.negy = fy && inv.y < 0.0f; r.negz = fz && inv.z < 0.0f;
    r.flat = (fx ? 0u : 1u) | (fy ? 0u : 2u) | (fz ? 0u : 4u);
    return r;
}

// intersect_box (intersect.h:113-157) from the ray's slab constants: a flat
// axis is skipped (the reference's isfinite test), the others compute
// fmaf(bound, inv, noid) exactly as intersect_box does.
__device__ __forceinline__ bool intersect_box_slab(const RaySlab &r, V3 lo, V3 hi, float &dist) {
    float tmin = 0.0f, tmax = __builtin_inff();
    if (!(r.flat & 1u)) {
        const float t0 = __builtin_fmaf(lo.x, r.inx, r.onx), t1 = __builtin_fmaf(hi.x, r.inx, r.onx);
        tmin = fmax_(tmin, fmin_(t0, t1)); tmax = fmin_(tmax, fmax_(t0, t1));
    }
    if (!(r.flat & 2u)) {
        const float t0 = __builtin_fmaf(lo.y, r.iny, r.ony), t1 = __builtin_fmaf(hi.y, r.iny, r.ony);
        tmin = fmax_(tmin, fmin_(t0, t1)); tmax = fmin_(tmax, fmax_(t0, t1));
    }
    if (!(r.flat & 4u)) {
        const float t0 = __builtin_fmaf(lo.z, r.inz, r.onz), t1 = __builtin_fmaf(hi.z, r.inz, r.onz);
        tmin = fmax_(tmin, fmin_(t0, t1)); tmax = fmin_(tmax, fmax_(t0, t1));
    }
    if (tmin > tmax) return false;
    dist = tmin;
    return true;
}

// The reference's nearest-hit decision (mesh.h:45-126) between a candidate X
// (Moller-Trumbore distance dx, reference DFS rank rx, entry distance bdx of its
// reference leaf box, which the ray hits) and the best so far B (db, rb, bdb;
// none: db = bdb = inf, rb = ~0).  The reference meets triangles in rank order,
// keeps the first, and replaces it only by a later one whose leaf box passes the
// prune (box entry <= the kept distance, mesh.h:94-96) and whose distance is
// strictly smaller:
//   rx > rb (B met first): X replaces B  iff  bdx <= db && dx < db;
//   rx < rb (X met first): B would not have replaced X unless bdb <= dx && db < dx.
// When every hit lies beyond its own box's entry (bd <= d) this is the
// (distance, rank) minimum of the earlier rounds.  It is not when the float
// Moller-Trumbore reports a hit BEFORE the box entry (a grazing triangle far
// away: the 29k bench's photon 9,043,377 hits a triangle at 36,510.26 mm whose
// leaf box the ray enters at 36,511.24; the exact ray misses that triangle
// triangle's plane 7% (in barycentrics) outside it), which the reference keeps
// when it meets it first.
__device__ __forceinline__ bool ref_may_beat(float dx, uint32_t rx, float db, uint32_t rb, float bdb) {
    return rx < rb ? !(bdb <= dx && db < dx) : dx < db;   // before X's leaf box is tested
}
__device__ __forceinline__ bool ref_beats(float dx, uint32_t rx, float bdx, float db, uint32_t rb, float bdb) {
    return rx < rb ? !(bdb <= dx && db < dx) : (bdx <= db && dx < db);
}
// Culling threshold for boxes: a triangle X can replace B only if dx <=
// max(db, bdb), and the boxes holding X are entered at most `undershoot` after
// dx.  The float false positives above undershoot by up to 2.5e-4 of the
// distance (5.8 mm) in 10 M photons of the 29k bench (oracle.undershoot): the
// traversal keeps every box entered within 2^-11 (4.9e-4) + 1 mm of
// max(db, bdb).  (inf stays inf: no best yet.)
#ifndef CHR_CUT_REL   // (build-time A/B of the margin: -DCHR_CUT_REL=0.0f -DCHR_CUT_ABS=0.0f)
#define CHR_CUT_REL 0x1p-11f
#endif
#ifndef CHR_CUT_ABS
#define CHR_CUT_ABS 1.0f
#endif
__device__ __forceinline__ float ref_cut(float db, float bdb) {
    const float m = __builtin_fmaxf(db, bdb);
    return __builtin_fmaf(m, CHR_CUT_REL, m + CHR_CUT_ABS);
}
// Two lanes' candidates (id -1: none, with d = bd = inf, rank = ~0) merged by the
// rule above (the one the reference meets first, unless the other replaces it):
// symmetric, so a butterfly leaves every lane of a segment with the same winner.
constexpr uint32_t NONE32 = 0xFFFFFFFFu;
struct RefHit {
    float d, bd;
    uint32_t rank;
    int id;
};
__device__ __forceinline__ RefHit ref_merge(const RefHit &a, const RefHit &b) {
    return ref_beats(b.d, b.rank, b.bd, a.d, a.rank, a.bd) ? b : a;
}
__device__ __forceinline__ RefHit shfl_xor_hit(const RefHit &h, int off) {
    return RefHit{__shfl_xor(h.d, off), __shfl_xor(h.bd, off), (uint32_t)__shfl_xor((int)h.rank, off),
                  __shfl_xor(h.id, off)};
}

// What a queued photon's walk is: 0 none (NaN state: the step aborts it,
// propagate.cu:307-310), 1 a walk.  (Rounds 2-4 had a kind 2, FLAT: a
// direction component with non-finite reciprocal, walked as 2^18 sub-walks;
// the flat-axis slab test above makes it an ordinary walk.)  d must be the
// normalised direction.
__device__ __forceinline__ int walk_kind(V3 o, V3 d) {
    const float prod = ((((d.x * d.y) * d.z) * o.x) * o.y) * o.z;
    return chr_isnan(prod) ? 0 : 1;
}
// a flat ray (diagnostic counts: detail.flat_walks)
__device__ __forceinline__ bool flat_ray(V3 d) {
    return !(chr_isfinite(1.0f / d.x) && chr_isfinite(1.0f / d.y) && chr_isfinite(1.0f / d.z));
}

// Slab-test the up-to-8 children of one wide node.  Returns the leaf children
// hit (bit mask), leaves the nearest hit inner child in near_node/near_t and
// pushes the other hit inner children in child order.  Boxes entered beyond
// `cut` (ref_cut of the best so far) are culled (strict '>', mesh.h:94-96).  Branch-free over the children
// (the per-child early-outs of a loop cost ~3 scalar exec-mask instructions
// each and divide the wave anyway): all 8 slab tests, the near child as the
// first of the smallest entry distance, then one predicated push per child at
// its prefix position.
template <int SL = WIDE_LDS, int TB = BLOCK>
__device__ __forceinline__ uint32_t expand_node(const uint4 h, const uint4 a1, const uint4 a2, const uint4 a3,
                                                const uint4 a4, const uint4 a5, const RaySlab &r, float cut,
                                                uint32_t &near_node, float &near_t, WStack &st, int &sp,
                                                uint32_t &overflow, uint32_t cmask = 0xFFu) {
    const V3 org = v3(__uint_as_float(h.x), __uint_as_float(h.y), __uint_as_float(h.z));
    const float sx = exp_scale(h.w), sy = exp_scale(h.w >> 8), sz = exp_scale(h.w >> 16);
    // byte arrays: x lo = a1.xy, y lo = a1.zw, z lo = a2.xy, x hi = a2.zw, y hi = a3.xy, z hi = a3.zw
    const uint32_t nx0 = r.negx ? a2.z : a1.x, nx1 = r.negx ? a2.w : a1.y;
    const uint32_t fx0 = r.negx ? a1.x : a2.z, fx1 = r.negx ? a1.y : a2.w;
    const uint32_t ny0 = r.negy ? a3.x : a1.z, ny1 = r.negy ? a3.y : a1.w;
    const uint32_t fy0 = r.negy ? a1.z : a3.x, fy1 = r.negy ? a1.w : a3.y;
    const uint32_t nz0 = r.negz ? a3.z : a2.x, nz1 = r.negz ? a3.w : a2.y;
    const uint32_t fz0 = r.negz ? a2.x : a3.z, fz1 = r.negz ? a2.y : a3.w;
    float tk[8];
    uint32_t inner = 0, leaf = 0;
    // two children per packed FMA (v_pk_fma_f32: each half a fused fmaf, so the
    // plane distances are bit-identical to the scalar form above)
    const F2 sx2 = f2(sx, sx), sy2 = f2(sy, sy), sz2 = f2(sz, sz);
    const F2 ox2 = f2(org.x, org.x), oy2 = f2(org.y, org.y), oz2 = f2(org.z, org.z);
    const F2 ix2 = f2(r.inx, r.inx), iy2 = f2(r.iny, r.iny), iz2 = f2(r.inz, r.inz);
    const F2 nx2 = f2(r.onx, r.onx), ny2 = f2(r.ony, r.ony), nz2 = f2(r.onz, r.onz);
    const F2 fx2 = f2(r.ofx, r.ofx), fy2 = f2(r.ofy, r.ofy), fz2 = f2(r.ofz, r.ofz);
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
        const F2 tnx = pk_fma(pk_fma(f2(byte_f(nx0, nx1, k), byte_f(nx0, nx1, k + 1)), sx2, ox2), ix2, nx2);
        const F2 tfx = pk_fma(pk_fma(f2(byte_f(fx0, fx1, k), byte_f(fx0, fx1, k + 1)), sx2, ox2), ix2, fx2);
        const F2 tny = pk_fma(pk_fma(f2(byte_f(ny0, ny1, k), byte_f(ny0, ny1, k + 1)), sy2, oy2), iy2, ny2);
        const F2 tfy = pk_fma(pk_fma(f2(byte_f(fy0, fy1, k), byte_f(fy0, fy1, k + 1)), sy2, oy2), iy2, fy2);
        const F2 tnz = pk_fma(pk_fma(f2(byte_f(nz0, nz1, k), byte_f(nz0, nz1, k + 1)), sz2, oz2), iz2, nz2);
        const F2 tfz = pk_fma(pk_fma(f2(byte_f(fz0, fz1, k), byte_f(fz0, fz1, k + 1)), sz2, oz2), iz2, fz2);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = k + h;
            const uint32_t kind = ((c < 4 ? a4.z : a4.w) >> (8 * (c & 3))) & 0xFFu;
            const float tmin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(tnx[h], tny[h]), tnz[h]), 0.0f);
            const float tmax = __builtin_fminf(__builtin_fminf(tfx[h], tfy[h]), tfz[h]);
            const bool hit = (kind != 0u) & (((cmask >> c) & 1u) != 0u) & !(tmin > tmax) & !(tmin > cut);
            inner |= (uint32_t)(hit & (kind == WIDE_INNER)) << c;
            leaf |= (uint32_t)(hit & (kind != WIDE_INNER)) << c;
            tk[c] = tmin;
        }
    }
    // nearest inner child: first of the smallest entry distance
    int nk = -1;
    float nt = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const bool take = ((inner >> k) & 1u) && (nk < 0 || tk[k] < nt);
        nk = take ? k : nk;
        nt = take ? tk[k] : nt;
    }
    near_node = 0xFFFFFFFFu;
    near_t = 0.0f;
    if (nk >= 0) {
        near_node = a4.x + (((nk < 4 ? a5.x : a5.y) >> (8 * (nk & 3))) & 0xFFu);
        near_t = nt;
    }
    const uint32_t push = nk >= 0 ? inner & ~(1u << nk) : 0u;
    if (push) {
        const int npush = __builtin_popcount(push);
        if (sp + npush < SL) {
            // all in LDS: every child writes, the ones not pushed to the slot above
            // the new top (free, so harmless) -- no per-child branch
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int pos = ((push >> k) & 1u) ? sp + __builtin_popcount(push & ((1u << k) - 1u)) : sp + npush;
                st.node[pos * TB] = a4.x + (((k < 4 ? a5.x : a5.y) >> (8 * (k & 3))) & 0xFFu);
                st.dist[pos * TB] = tk[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int pos = sp + __builtin_popcount(push & ((1u << k) - 1u));
                if (((push >> k) & 1u) && pos < WIDE_STACK)
                    wpush<SL, TB>(st, pos, a4.x + (((k < 4 ? a5.x : a5.y) >> (8 * (k & 3))) & 0xFFu), tk[k]);
            }
        }
        if (sp + npush > WIDE_STACK) {
            overflow += (uint32_t)(sp + npush - WIDE_STACK);
            sp = WIDE_STACK;
        } else {
            sp += npush;
        }
    }
    return leaf;
}

struct WalkCounts {   // filled only by the counting variant (bench: algorithmic bytes per photon)
    uint32_t nodes, tris, walks;
    uint32_t wave_nodes, wave_tris;   // steps the whole wave executed (counted by its first active lane)
    unsigned long long wave_fill_cycles, wave_other_cycles;   // s_memtime spent in fill_state / rest of the step loop
    uint32_t flat;                    // flat walks (walk_kind 2) walked whole (group walk; always counted)
};
__device__ __forceinline__ bool wave_leader() {
    const unsigned long long m = __ballot(1);
    return (unsigned)__lane_id() == (unsigned)(__ffsll((long long)m) - 1);
}

// ---------------------------------------------------------------- device profile
// The reference's CHROMA_DEVICE_PROFILE regions (profile.h:9-37: per-call
// clock64 spans atomically added to per-region counters) for the split step
// kernels, built only into libchroma_amd_prof.so (-DCHR_DEVICE_PROFILE=1).
// Instead of two global atomics per call, each work-item keeps its region
// lane-cycles and calls in registers and a wave adds its sums once at exit.
// A kernel marks region boundaries with tick(next): the wave time since the
// last tick goes to the region the work-item was in (a work-item masked off in
// a branch keeps its region, so the time it waits is charged there).
#ifdef CHR_DEVICE_PROFILE
__device__ unsigned long long chr_prof_calls[CHR_PROF_COUNT];
__device__ unsigned long long chr_prof_cycles[CHR_PROF_COUNT];

// one wave's sum of (calls, cycles) added to region id; every lane of the wave active
__device__ __forceinline__ void prof_add(int id, unsigned long long calls, unsigned long long cycles) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        calls += __shfl_xor(calls, o);
        cycles += __shfl_xor(cycles, o);
    }
    if (__lane_id() == 0) {
        if (calls) atomicAdd(&chr_prof_calls[id], calls);
        if (cycles) atomicAdd(&chr_prof_cycles[id], cycles);
    }
}
template <int N>
struct Prof {
    uint32_t cyc[N], calls[N];
    unsigned long long t, t0;
    int cur;
    __device__ __forceinline__ void start(int c) {
        t0 = t = __builtin_amdgcn_s_memtime();
        cur = c;
#pragma unroll
        for (int i = 0; i < N; ++i) cyc[i] = calls[i] = 0u;
    }
    __device__ __forceinline__ void tick(int next) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        const uint32_t dt = (uint32_t)(now - t);
        t = now;
#pragma unroll
        for (int i = 0; i < N; ++i) cyc[i] += cur == i ? dt : 0u;
        cur = next;
    }
    __device__ __forceinline__ void set(int c) { cur = c; }
    __device__ __forceinline__ void call(int i, uint32_t k = 1u) { calls[i] += k; }
    __device__ __forceinline__ unsigned long long total() const { return t - t0; }
};
#else
template <int N>
struct Prof {
    __device__ __forceinline__ void start(int) {}
    __device__ __forceinline__ void tick(int) {}
    __device__ __forceinline__ void set(int) {}
    __device__ __forceinline__ void call(int, uint32_t = 1u) {}
};
#endif

// Photon watch (profile build only, chr_watch_set / chr_watch_fetch): every step
// of one photon (its index in one batch's arrays) recorded by the kernel that ran
// it, in the layout of the oracle's orc_set_watch, so a parity mismatch can be
// followed step by step on both sides.  Words: kind (1 shade, 2 tail), queue
// position, hit triangle (-1: none), walk distance, pos in (3), dir in (3), last
// hit in, material1, absorption length, scattering length, pos out (3), history
// out, time out, RNG slot.
#ifdef CHR_DEVICE_PROFILE
constexpr uint32_t CHR_WATCH_WORDS = 20, CHR_WATCH_MAX = 4096;
__device__ uint32_t chr_watch_pid = 0xFFFFFFFFu;
__device__ unsigned long long chr_watch_array = 0ull;   // the batch's pos array (0: any batch)
__device__ uint32_t chr_watch_n = 0u;
__device__ uint32_t chr_watch_buf[CHR_WATCH_MAX * CHR_WATCH_WORDS];
struct Watch {
    uint32_t w[CHR_WATCH_WORDS];
    bool on;
    __device__ __forceinline__ void begin(uint32_t kind, uint32_t pid, const float *pos_array, uint32_t q,
                                          uint32_t slot, V3 pos, V3 dir, int last_in) {
        on = chr_watch_pid != 0xFFFFFFFFu && pid == chr_watch_pid && (chr_watch_array == 0ull || chr_watch_array == (unsigned long long)pos_array);
        if (!on) return;
        w[0] = kind; w[1] = q; w[19] = slot;
        w[4] = __float_as_uint(pos.x); w[5] = __float_as_uint(pos.y); w[6] = __float_as_uint(pos.z);
        w[7] = __float_as_uint(dir.x); w[8] = __float_as_uint(dir.y); w[9] = __float_as_uint(dir.z);
        w[10] = (uint32_t)last_in;
    }
    __device__ __forceinline__ void filled(int tri, const State &s) {
        if (!on) return;
        w[2] = (uint32_t)tri; w[3] = __float_as_uint(s.distance); w[11] = (uint32_t)s.material1;
        w[12] = __float_as_uint(s.absorption_length); w[13] = __float_as_uint(s.scattering_length);
    }
    __device__ __forceinline__ void end(V3 pos, uint32_t history, float time) {
        if (!on) return;
        w[14] = __float_as_uint(pos.x); w[15] = __float_as_uint(pos.y); w[16] = __float_as_uint(pos.z);
        w[17] = history; w[18] = __float_as_uint(time);
        const uint32_t i = atomicAdd(&chr_watch_n, 1u);
        if (i < CHR_WATCH_MAX)
            for (uint32_t k = 0; k < CHR_WATCH_WORDS; ++k) chr_watch_buf[i * CHR_WATCH_WORDS + k] = w[k];
        on = false;
    }
};
// trace_kernel's walk of the watched ray (origin bits chr_wray_o, chr_watch_ray):
// one 8-word event per step of its lane -- kind, then kind-specific words.
constexpr uint32_t CHR_WEV_MAX = 8192;
__device__ uint32_t chr_wray_on = 0u;
__device__ uint32_t chr_wray_o[3];
__device__ uint32_t chr_wev_n = 0u;
__device__ uint32_t chr_wev_buf[CHR_WEV_MAX * 8];
__device__ __forceinline__ bool wray_match(V3 o) {
    return chr_wray_on && __float_as_uint(o.x) == chr_wray_o[0] && __float_as_uint(o.y) == chr_wray_o[1] &&
           __float_as_uint(o.z) == chr_wray_o[2];
}
__device__ __forceinline__ void wev(uint32_t k, uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e,
                                    uint32_t f, uint32_t h) {
    const uint32_t i = atomicAdd(&chr_wev_n, 1u);
    if (i >= CHR_WEV_MAX) return;
    uint32_t *w = chr_wev_buf + 8 * i;
    w[0] = k; w[1] = a; w[2] = b; w[3] = c; w[4] = d; w[5] = e; w[6] = f; w[7] = h;
}
#define CHR_WEV(on, ...) do { if (on) wev(__VA_ARGS__); } while (0)
#else
#define CHR_WEV(on, ...) do { } while (0)
struct Watch {
    __device__ __forceinline__ void begin(uint32_t, uint32_t, const float *, uint32_t, uint32_t, V3, V3, int) {}
    __device__ __forceinline__ void filled(int, const State &) {}
    __device__ __forceinline__ void end(V3, uint32_t, float) {}
};
#endif

// The same query, scheduled for 64-wide SIMT (default).  Leaf triangles are
// not tested inside the node step of the lane that reached them: a lane that
// hits leaves parks them (one node's worth) and the WAVE decides each
// iteration, by ballot, between a node step (lanes without parked work) and
// a triangle step (every lane with parked work tests one triangle) -- the
// triangle step runs when >= TRI_BATCH lanes have work or no lane can
// traverse.  This keeps most lanes busy in both kinds of step (measured
// SIMD efficiency of the per-node loop above: 6% for triangles).
// Moller-Trumbore runs first; the reference leaf slab test + prune
// (mesh.h:94-96) is evaluated only for a hit that would become the best,
// with the same `best`, so the accept decision is unchanged.
template <bool COUNT, int TRI_BATCH>
__device__ int intersect_wide_sched(const DevGeom &g, V3 o, V3 d, float &min_distance, int last_hit, WStack &st,
                                    uint32_t &overflow, WalkCounts &cnt) {
    if constexpr (COUNT) cnt.walks++;
    const V3 noid = v3(-o.x / d.x, -o.y / d.y, -o.z / d.z);
    const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const RaySlab slab = make_slab(o, noid, inv);
    float best = __builtin_inff(), best_bd = __builtin_inff(), cut = __builtin_inff();
    uint32_t best_rank = 0xFFFFFFFFu;
    int best_id = -1;
    const uint32_t last = (uint32_t)last_hit;
    int sp = 0;
    uint32_t node = 0;              // node to expand next (INVALID: pop)
    bool done = false;
    // parked leaf work of one node: current leaf [pcur, pcur+pleft), further hit leaves in pmask
    uint32_t pcur = 0, pleft = 0, pmask = 0, pbase = 0;
    unsigned long long pkinds = 0, poffs = 0;
    constexpr uint32_t INVALID = 0xFFFFFFFFu;
    while (true) {
        const bool has_work = pleft != 0;
        const bool can_walk = !done && !has_work;
        const unsigned long long mw = __ballot(can_walk);
        const unsigned long long mt = __ballot(has_work);
        if ((mw | mt) == 0) break;
        // TRI_BATCH == 0: no wave-level choice -- every iteration each lane
        // does whichever step it has (parked triangle first)
        if (TRI_BATCH == 0 ? can_walk : (mw != 0 && __popcll(mt) < TRI_BATCH)) {
            // ------------------------------------------------ node step
            if (!can_walk) continue;
            if (node == INVALID) {
                bool found = false;
                while (sp > 0) {
                    sp--;
                    float t;
                    wpop(st, sp, node, t);
                    if (!(t > cut)) { found = true; break; }
                }
                if (!found) { done = true; continue; }
            }
            if constexpr (COUNT) { cnt.nodes++; if (wave_leader()) cnt.wave_nodes++; }
            const uint4 *np = g.wnodes + (size_t)g.wstride * node;
            const uint4 h = gld(np), a1 = gld(np + 1), a2 = gld(np + 2), a3 = gld(np + 3), a4 = gld(np + 4),
                        a5 = gld(np + 5);
            uint32_t near_node;
            float near_t;
            const uint32_t leaf_mask =
                expand_node(h, a1, a2, a3, a4, a5, slab, cut, near_node, near_t, st, sp, overflow);
            node = near_node;
            if (leaf_mask) {
                pkinds = ((unsigned long long)a4.w << 32) | a4.z;
                poffs = ((unsigned long long)a5.y << 32) | a5.x;
                pbase = a4.y;
                const int k = __builtin_ctz(leaf_mask);
                pmask = leaf_mask & (leaf_mask - 1);
                pleft = (uint32_t)(pkinds >> (8 * k)) & 0xFFu;
                pcur = pbase + ((uint32_t)(poffs >> (8 * k)) & 0xFFu);
            }
        } else {
            // ------------------------------------------------ triangle step
            if (!has_work) continue;
            if constexpr (COUNT) { cnt.tris++; if (wave_leader()) cnt.wave_tris++; }
            const float4 *r = g.wtri + 4 * (size_t)pcur;
            const float4 r0 = gld(r), r1 = gld(r + 1), r2 = gld(r + 2);
            pcur++;
            if (--pleft == 0 && pmask) {
                const int k = __builtin_ctz(pmask);
                pmask &= pmask - 1;
                pleft = (uint32_t)(pkinds >> (8 * k)) & 0xFFu;
                pcur = pbase + ((uint32_t)(poffs >> (8 * k)) & 0xFFu);
            }
            const uint32_t id = __float_as_uint(r2.y);
            float dist;
            if (id == last ||
                !intersect_record(o, d, r0, r1, r2, dist))
                continue;
            const uint32_t rank = __float_as_uint(r2.z);
            if (!ref_may_beat(dist, rank, best, best_rank, best_bd)) continue;
            const float4 r3 = gld(r + 3);
            V3 lo, hi;
            node_bounds(g, make_uint4(__float_as_uint(r2.w), __float_as_uint(r3.x), __float_as_uint(r3.y), 0u), lo, hi);
            float bd;
            if (!intersect_box(noid, inv, lo, hi, bd) || !ref_beats(dist, rank, bd, best, best_rank, best_bd))
                continue;   // mesh.h:94-96
            best = dist;
            best_rank = rank;
            best_bd = bd;
            cut = ref_cut(best, best_bd);
            best_id = rec_of(g, r);
        }
    }
    min_distance = best_id == -1 ? -1.0f : best;
    return best_id;
}

// Speculative variant of the scheduled walk (Aila & Laine 2009, "speculative
// traversal"): a lane that reaches leaves parks them in a small LDS queue and
// keeps walking (with the best it has so far) while the queue has room for a
// node's worth of leaves; the WAVE runs a triangle step only once at least
// F/8 of its live lanes have parked triangles (or no lane can walk), so the
// triangle steps run with most lanes busy instead of a handful.  Each lane
// still tests its own triangles in the order it found them, with the accept
// rule and reference leaf check of intersect_wide_sched; walking ahead with a
// best that is not yet updated only adds nodes/triangles to what is tested
// (a superset: culling uses a best that never drops below the final one), so
// the nearest hit is unchanged.
// Leaf queue entry: first triangle record (bits 0-29) | (count-1) << 30.
template <bool COUNT, int F>
__device__ int intersect_wide_spec(const DevGeom &g, V3 o, V3 d, float &min_distance, int last_hit, WStack &st,
                                   uint32_t &overflow, WalkCounts &cnt) {
    if constexpr (COUNT) cnt.walks++;
    const V3 noid = v3(-o.x / d.x, -o.y / d.y, -o.z / d.z);
    const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const RaySlab slab = make_slab(o, noid, inv);
    float best = __builtin_inff(), best_bd = __builtin_inff(), cut = __builtin_inff();
    uint32_t best_rank = 0xFFFFFFFFu;
    int best_id = -1;
    const uint32_t last = (uint32_t)last_hit;
    int sp = 0;
    uint32_t node = 0;
    bool done = false;
    uint32_t qh = 0, qt = 0;        // queue head / tail (free-running; slot = x % LEAFQ)
    uint32_t pcur = 0, pleft = 0;   // leaf being tested
    constexpr uint32_t INVALID = 0xFFFFFFFFu;
    while (true) {
        const bool has_work = pleft != 0 || qh != qt;
        const bool can_walk = !done && (qt - qh) <= (uint32_t)(LEAFQ - 8);
        const unsigned long long mw = __ballot(can_walk);
        const unsigned long long mt = __ballot(has_work);
        if ((mw | mt) == 0) break;
        if (mw != 0 && 8 * __popcll(mt) < F * __popcll(mw | mt)) {
            // ------------------------------------------------ node step
            if (!can_walk) continue;
            if (node == INVALID) {
                bool found = false;
                while (sp > 0) {
                    sp--;
                    float t;
                    wpop(st, sp, node, t);
                    if (!(t > cut)) { found = true; break; }
                }
                if (!found) { done = true; continue; }
            }
            if constexpr (COUNT) { cnt.nodes++; if (wave_leader()) cnt.wave_nodes++; }
            const uint4 *np = g.wnodes + (size_t)g.wstride * node;
            const uint4 h = gld(np), a1 = gld(np + 1), a2 = gld(np + 2), a3 = gld(np + 3), a4 = gld(np + 4),
                        a5 = gld(np + 5);
            uint32_t near_node;
            float near_t;
            uint32_t leaf_mask = expand_node(h, a1, a2, a3, a4, a5, slab, cut, near_node, near_t, st, sp, overflow);
            node = near_node;
            while (leaf_mask) {
                const int k = __builtin_ctz(leaf_mask);
                leaf_mask &= leaf_mask - 1;
                const uint32_t kind = ((k < 4 ? a4.z : a4.w) >> (8 * (k & 3))) & 0xFFu;
                const uint32_t first = a4.y + (((k < 4 ? a5.x : a5.y) >> (8 * (k & 3))) & 0xFFu);
                st.leafq[(qt % LEAFQ) * BLOCK] = first | ((kind - 1u) << 30);
                qt++;
            }
        } else {
            // ------------------------------------------------ triangle step
            if (!has_work) continue;
            if (pleft == 0) {
                const uint32_t e = st.leafq[(qh % LEAFQ) * BLOCK];
                qh++;
                pcur = e & 0x3FFFFFFFu;
                pleft = (e >> 30) + 1u;
            }
            if constexpr (COUNT) { cnt.tris++; if (wave_leader()) cnt.wave_tris++; }
            const float4 *r = g.wtri + 4 * (size_t)pcur;
            const float4 r0 = gld(r), r1 = gld(r + 1), r2 = gld(r + 2);
            pcur++;
            pleft--;
            const uint32_t id = __float_as_uint(r2.y);
            float dist;
            if (id == last ||
                !intersect_record(o, d, r0, r1, r2, dist))
                continue;
            const uint32_t rank = __float_as_uint(r2.z);
            if (!ref_may_beat(dist, rank, best, best_rank, best_bd)) continue;
            const float4 r3 = gld(r + 3);
            V3 lo, hi;
            node_bounds(g, make_uint4(__float_as_uint(r2.w), __float_as_uint(r3.x), __float_as_uint(r3.y), 0u), lo, hi);
            float bd;
            if (!intersect_box(noid, inv, lo, hi, bd) || !ref_beats(dist, rank, bd, best, best_rank, best_bd))
                continue;   // mesh.h:94-96
            best = dist;
            best_rank = rank;
            best_bd = bd;
            cut = ref_cut(best, best_bd);
            best_id = rec_of(g, r);
        }
    }
    min_distance = best_id == -1 ? -1.0f : best;
    return best_id;
}

__device__ __forceinline__ uint32_t byte_of(uint32_t lo4, uint32_t hi4, int k) {
    return ((k < 4 ? lo4 : hi4) >> (8 * (k & 3))) & 0xFFu;
}

// ---------------------------------------------------------------- photon.h
__device__ __forceinline__ int convert(int c) { return (c & 0x80) ? (int)(0xFFFFFF00u | (uint32_t)c) : c; }
__device__ __forceinline__ float get_theta(V3 a, V3 b) { return chr_acosf(fmax_(-1.0f, fmin_(1.0f, dot(a, b)))); }

// analytic wire planes (photon.h:108-270), FP64, rare path
__device__ CHR_COLD void wireplanes(const DevGeom &g, const Photon &p, float best_distance, int &a_surface,
                                        int &a_inner, int &a_outer, V3 &a_normal_raw, float &a_dot_raw,
                                        float &a_distance) {
    for (int ip = 0; ip < (int)g.nwireplanes; ++ip) {
        const chr_wireplane_desc &wp = g.wireplanes[ip];
        const double ux = wp.u[0], uy = wp.u[1], uz = wp.u[2];
        const double vx0 = wp.v[0], vy0 = wp.v[1], vz0 = wp.v[2];
        const double un = 1.0 / sqrt(ux * ux + uy * uy + uz * uz);
        const double ux1 = ux * un, uy1 = uy * un, uz1 = uz * un;
        const double vdotu = vx0 * ux1 + vy0 * uy1 + vz0 * uz1;
        const double vx1 = vx0 - vdotu * ux1, vy1 = vy0 - vdotu * uy1, vz1 = vz0 - vdotu * uz1;
        const double vn = 1.0 / sqrt(vx1 * vx1 + vy1 * vy1 + vz1 * vz1);
        const double vx = vx1 * vn, vy = vy1 * vn, vz = vz1 * vn;
        const double nx = uy1 * vz - uz1 * vy, ny = uz1 * vx - ux1 * vz, nz = ux1 * vy - uy1 * vx;
        const V3 w = p.pos - v3(wp.origin[0], wp.origin[1], wp.origin[2]);
        const double du = (double)p.dir.x * ux1 + (double)p.dir.y * uy1 + (double)p.dir.z * uz1;
        const double dv = (double)p.dir.x * vx + (double)p.dir.y * vy + (double)p.dir.z * vz;
        const double dn = (double)p.dir.x * nx + (double)p.dir.y * ny + (double)p.dir.z * nz;
        const double wu = (double)w.x * ux1 + (double)w.y * uy1 + (double)w.z * uz1;
        const double wv0 = (double)w.x * vx + (double)w.y * vy + (double)w.z * vz - (double)wp.v0;
        const double wn0 = (double)w.x * nx + (double)w.y * ny + (double)w.z * nz;
        double t_in = -1.0e300, t_out = 1.0e300;
        if (fabs(du) < 1e-15) {
            if (wu < (double)wp.umin || wu > (double)wp.umax) continue;
        } else {
            double t1 = ((double)wp.umin - wu) / du, t2 = ((double)wp.umax - wu) / du;
            if (t1 > t2) { double tmp = t1; t1 = t2; t2 = tmp; }
            if (t1 > t_in) t_in = t1;
            if (t2 < t_out) t_out = t2;
            if (t_in > t_out) continue;
        }
        const double pitch = (double)wp.pitch;
        const double inv_pitch = (pitch != 0.0) ? (1.0 / pitch) : 0.0;
        const double wire_radius = (double)wp.radius;
        const double wire_thickness = 2.0 * wire_radius;
        const double pad_v = 0.5 * wire_thickness + 1e-6, pad_n = 0.5 * wire_thickness + 1e-6;
        const int kmin = (int)ceil(((double)wp.vmin - (double)wp.v0) / pitch);
        const int kmax = (int)floor(((double)wp.vmax - (double)wp.v0) / pitch);
        const double A = dv * dv + dn * dn;
        int k_start = kmin, k_stop = kmax;
        if (kmin <= kmax) {
            const double t_eps = 1.0e-4;
            double t_lo = fmax(t_in, t_eps), t_hi = t_out;
            const double best_cap = (double)best_distance;
            if (best_cap < t_hi) t_hi = best_cap;
            if (fabs(dn) > 1e-12) {
                double tn1 = (-pad_n - wn0) / dn, tn2 = (pad_n - wn0) / dn;
                if (tn1 > tn2) { double tmp = tn1; tn1 = tn2; tn2 = tmp; }
                t_lo = fmax(t_lo, tn1); t_hi = fmin(t_hi, tn2);
            } else if (fabs(wn0) > pad_n) continue;
            if (t_hi < t_lo) continue;
            if (fabs(dn) <= 1e-12 && fabs(dv) > 1e-12) {
                const double t_span = (pitch + wire_thickness) / fabs(dv);
                t_hi = fmin(t_hi, t_lo + t_span);
            }
            const double v_entry = wv0 + dv * t_lo, v_exit = wv0 + dv * t_hi;
            double v_lo = fmin(v_entry, v_exit) - pad_v, v_hi = fmax(v_entry, v_exit) + pad_v;
            if (wv0 - pad_v < v_lo) v_lo = wv0 - pad_v;
            if (wv0 + pad_v > v_hi) v_hi = wv0 + pad_v;
            long long k_lo = (long long)floor(v_lo * inv_pitch), k_hi = (long long)ceil(v_hi * inv_pitch);
            if (k_lo < kmin) k_lo = kmin;
            if (k_hi > kmax) k_hi = kmax;
            if (k_lo > k_hi) continue;
            k_start = (int)k_lo; k_stop = (int)k_hi;
        }
        for (int k = k_start; k <= k_stop; ++k) {
            const double wv = wv0 - (double)k * pitch;
            const double B = wv * dv + wn0 * dn;
            const double C = wv * wv + wn0 * wn0 - wire_radius * wire_radius;
            const double disc = B * B - A * C;
            if (disc < 0.0) continue;
            const double sq = sqrt(disc);
            const double t_small = (-B - sq) / A, t_large = (-B + sq) / A;
            const double t_min = 1.0e-4;
            const double r2_wire = wire_radius * wire_radius;
            const double r2_0 = wv * wv + wn0 * wn0;
            const double eps0 = fmax(1e-18, 1e-12 * r2_wire);
            double t;
            if (r2_0 > r2_wire + eps0) { if (t_small <= t_min) continue; t = t_small; }
            else if (r2_0 < r2_wire - eps0) { if (t_large <= t_min) continue; t = t_large; }
            else t = t_min;
            const double uc = wu + du * t;
            if (uc < wp.umin || uc > wp.umax) continue;
            if ((float)t >= a_distance) continue;
            if (t < t_in || t > t_out) continue;
            const double vn_hit = wv + dv * t, nn_hit = wn0 + dn * t;
            const double len = sqrt(vn_hit * vn_hit + nn_hit * nn_hit);
            if (len <= 0.0) continue;
            const V3 nl = v3((float)((vn_hit / len) * vx + (nn_hit / len) * nx),
                             (float)((vn_hit / len) * vy + (nn_hit / len) * ny),
                             (float)((vn_hit / len) * vz + (nn_hit / len) * nz));
            a_distance = (float)t;
            a_surface = wp.surface_index;
            a_inner = wp.material_inner_index;
            a_outer = wp.material_outer_index;
            a_normal_raw = nl;
            a_dot_raw = dot(nl, -p.dir);
        }
    }
}

// Second half of fill_state (photon.h:272-397): the mesh hit (or an analytic
// wire plane, FP64) -> material pair, surface, oriented normal and the four
// interpolated bulk properties; no hit -> NO_HIT.  s.distance holds the mesh
// hit distance on entry.  REC: mesh_triangle is a wide-BVH triangle record
// (what the wide walks return: triangle id and vertices read from it); else a
// triangle id of the reference walk (the 48-byte reference records).
// WIRES = false: instantiated for geometries without analytic wire planes (the
// FP64 wire-plane code is then not part of the kernel at all)
template <bool REC, bool WIRES = true>
__device__ __forceinline__ void finish_fill(const DevGeom &g, State &s, Photon &p, int mesh_triangle) {
    int m1, m2;
    bool use_analytic = false;
    int a_surface = -1, a_inner = -1, a_outer = -1;
    V3 a_normal_raw = v3(0.0f, 0.0f, 0.0f);
    float a_dot_raw = 0.0f, a_distance = 1e30f;
    if (WIRES && g.nwireplanes > 0) {
        const float best_distance = (mesh_triangle == -1) ? 1e30f : s.distance;
        wireplanes(g, p, best_distance, a_surface, a_inner, a_outer, a_normal_raw, a_dot_raw, a_distance);
        if (a_surface >= 0) use_analytic = ((double)a_distance + 1e-12 < (double)best_distance);
    }
    if (use_analytic) {
        s.distance = a_distance;
        s.surface_index = a_surface;
        p.last_hit = -2;
        if (a_dot_raw > 0.0f) { m1 = a_outer; m2 = a_inner; s.normal = a_normal_raw; s.inside_to_outside = false; }
        else { m1 = a_inner; m2 = a_outer; s.normal = -a_normal_raw; s.inside_to_outside = true; }
    } else if (mesh_triangle != -1) {
        V3 e1, e3;   // v1 - v0, v2 - v1 (photon.h:365-367)
        int tid;
        uint32_t code;
        if constexpr (REC) {   // one record, four independent loads (no dependent material-code gather)
            const float4 *r = g.wtri + 4 * (size_t)mesh_triangle;
            const float4 r0 = gld(r), r1 = gld(r + 1), r2 = gld(r + 2), r3 = gld(r + 3);
            const V3 v0 = v3(r0.x, r0.y, r0.z), v1 = v3(r0.w, r1.x, r1.y), v2 = v3(r1.z, r1.w, r2.x);
            e1 = v1 - v0;
            e3 = v2 - v1;
            tid = (int)__float_as_uint(r2.y);
            code = __float_as_uint(r3.z);
        } else {
            const float4 *r = g.tri + 3 * (size_t)mesh_triangle;
            const float4 r0 = gld(r), r1 = gld(r + 1), r2 = gld(r + 2);
            e1 = v3(r0.w, r1.x, r1.y);
            e3 = v3(r2.y, r2.z, r2.w);
            tid = mesh_triangle;
            code = gld(g.material_codes + tid);
        }
        p.last_hit = tid;
        const int inner = convert(0xFF & (int)(code >> 24));
        const int outer = convert(0xFF & (int)(code >> 16));
        s.surface_index = convert(0xFF & (int)(code >> 8));
        s.normal = normalize(cross(e1, e3));
        if (dot(s.normal, -p.dir) > 0.0f) { m1 = outer; m2 = inner; s.inside_to_outside = false; }
        else { m1 = inner; m2 = outer; s.normal = -s.normal; s.inside_to_outside = true; }
    } else {
        p.last_hit = -1;
        p.history |= CHR_NO_HIT;
        return;
    }
    const DevMaterial &mat1 = g.materials[m1];
    const DevMaterial &mat2 = g.materials[m2];
    s.n1 = interp_property(g, p.wavelength, g.tables + mat1.refractive_index);
    s.n2 = interp_property(g, p.wavelength, g.tables + mat2.refractive_index);
    s.absorption_length = interp_property(g, p.wavelength, g.tables + mat1.absorption_length);
    s.scattering_length = interp_property(g, p.wavelength, g.tables + mat1.scattering_length);
    s.material1 = m1;
}

// photon.h:87-397
template <int BATCH, int WIDE, bool COUNT>
__device__ __forceinline__ void fill_state(const DevGeom &g, State &s, Photon &p, Stack st, WStack &wst,
                                           uint32_t &overflow, WalkCounts &cnt) {
    int mesh_triangle;
    if constexpr (WIDE >= 2000)   // speculative walk, triangle-step threshold (WIDE - 2000)/8 of live lanes
        mesh_triangle =
            intersect_wide_spec<COUNT, WIDE - 2000>(g, p.pos, p.dir, s.distance, p.last_hit, wst, overflow, cnt);
    else if constexpr (WIDE >= 1000)   // scheduled walk, triangle batch threshold WIDE - 1000
        mesh_triangle =
            intersect_wide_sched<COUNT, WIDE - 1000>(g, p.pos, p.dir, s.distance, p.last_hit, wst, overflow, cnt);
    else mesh_triangle = intersect_mesh<BATCH>(g, p.pos, p.dir, s.distance, p.last_hit, st, overflow);
    finish_fill<(WIDE != 0)>(g, s, p, mesh_triangle);
}

// photon.h:399-427
__device__ __forceinline__ V3 pick_new_direction(V3 axis, float theta, float phi) {
    float st, ct, sp, cp;
    chr_sincosf(theta, &st, &ct);
    chr_sincosf(phi, &sp, &cp);
    const float sat = chr_sqrtf(__builtin_fmaf(-axis.z, axis.z, 1.0f));
    float cap, sap;
    if (chr_isnan(sat) || sat < 0.00001f) { cap = 1.0f; sap = 0.0f; }
    else { cap = axis.x / sat; sap = axis.y / sat; }
    const float dx = __builtin_fmaf(st, __builtin_fmaf(axis.z * cp, cap, -(sp * sap)), ct * axis.x);
    const float dy = __builtin_fmaf(st, __builtin_fmaf(cp * axis.z, sap, sp * cap), ct * axis.y);
    const float dz = __builtin_fmaf(-(st * cp), sat, ct * axis.z);
    return v3(dx, dy, dz);
}

// photon.h:429-453
__device__ __forceinline__ void rayleigh_scatter(Photon &p, chr_xorwow &rng) {
    const float u = chr_uniform01(&rng);
    float cos_theta = 2.0f * chr_cosf((chr_acosf(__builtin_fmaf(-2.0f, u, 1.0f)) - 2 * PI_F) / 3.0f);
    if (cos_theta > 1.0f) cos_theta = 1.0f;
    else if (cos_theta < -1.0f) cos_theta = -1.0f;
    const float theta = chr_acosf(cos_theta);
    const float phi = chr_uniform(&rng, 0.0f, 2.0f * PI_F);
    p.dir = pick_new_direction(p.pol, theta, phi);
    if (1.0f - chr_fabsf(cos_theta) < 1e-6f)
        p.pol = pick_new_direction(p.pol, PI_F / 2.0f, phi);
    else
        p.pol = v3(__builtin_fmaf(-cos_theta, p.dir.x, p.pol.x), __builtin_fmaf(-cos_theta, p.dir.y, p.pol.y),
                   __builtin_fmaf(-cos_theta, p.dir.z, p.pol.z));
    p.dir = p.dir / norm(p.dir);
    p.pol = p.pol / norm(p.pol);
}

// photon.h:455-570
__device__ __forceinline__ int propagate_to_boundary(const DevGeom &g, Photon &p, State &s, chr_xorwow &rng, int use_weights,
                                     int scatter_first) {
    float absorption_distance = -s.absorption_length * chr_logf(chr_uniform01(&rng));
    float scattering_distance = -s.scattering_length * chr_logf(chr_uniform01(&rng));
    if (use_weights && p.weight > WEIGHT_LOWER_THRESHOLD) absorption_distance = 1e30f;
    else use_weights = 0;
    if (scatter_first == 1) {
        const float scatter_prob = 1.0f - chr_expf(-s.distance / s.scattering_length);
        if (scatter_prob > WEIGHT_LOWER_THRESHOLD) {
            int i = 0;
            while (i < 1000 && scattering_distance > s.distance) {
                scattering_distance = -s.scattering_length * chr_logf(chr_uniform01(&rng));
                i++;
            }
            p.weight *= scatter_prob;
        }
    } else if (scatter_first == -1) {
        const float no_scatter_prob = chr_expf(-s.distance / s.scattering_length);
        if (no_scatter_prob > WEIGHT_LOWER_THRESHOLD) {
            int i = 0;
            while (i < 1000 && scattering_distance <= s.distance) {
                scattering_distance = -s.scattering_length * chr_logf(chr_uniform01(&rng));
                i++;
            }
            p.weight *= no_scatter_prob;
        }
    }
    if (absorption_distance <= scattering_distance) {
        if (absorption_distance <= s.distance) {
            p.time = p.time + absorption_distance / (SPEED_OF_LIGHT / s.n1);
            p.pos = axpy(absorption_distance, p.dir, p.pos);
            const DevMaterial &m = g.materials[s.material1];
            if (m.num_comp == 0) {
                p.last_hit = -1;
                p.history |= CHR_BULK_ABSORB;
                return BREAK;
            }
            const uint32_t W1 = g.wl_n + 1, T1 = g.t_n + 1;
            const float usc = chr_uniform01(&rng);
            float prob = 0.0f;
            uint32_t comp;
            for (comp = 0;; comp++) {
                const float comp_abs = interp_property(g, p.wavelength, g.tables + m.comp_absorption_length + comp * W1);
                prob += s.absorption_length / comp_abs;
                if (usc < prob || comp + 1 == m.num_comp) break;
            }
            const float usr = chr_uniform01(&rng);
            const float crp = interp_property(g, p.wavelength, g.tables + m.comp_reemission_prob + comp * W1);
            if (usr < crp) {
                p.wavelength = sample_cdf(rng, (int)g.wl_n, g.wl_start, g.wl_step,
                                          g.tables + m.comp_reemission_wvl_cdf + comp * W1);
                const float *tcdf = g.tables_g + m.comp_reemission_time_cdf + comp * T1;
                if (m.comp_time_index != ~0u)
                    p.time += sample_cdf_indexed(rng, g.t_start, g.t_step, tcdf,
                                                 (const uint32_t *)g.tables_g + m.comp_time_index +
                                                     comp * (TIME_INDEX_BUCKETS + 1),
                                                 TIME_INDEX_BUCKETS);
                else
                    p.time += sample_cdf(rng, (int)g.t_n, g.t_start, g.t_step, tcdf);
                p.dir = uniform_sphere(rng);
                p.pol = cross(uniform_sphere(rng), p.dir);
                p.pol = p.pol / norm(p.pol);
                p.last_hit = -1;
                p.history |= CHR_BULK_REEMIT;
                return CONTINUE;
            }
            p.last_hit = -1;
            p.history |= CHR_BULK_ABSORB;
            return BREAK;
        }
    } else {
        if (scattering_distance <= s.distance) {
            if (use_weights) p.weight *= chr_expf(-scattering_distance / s.absorption_length);
            p.time = p.time + scattering_distance / (SPEED_OF_LIGHT / s.n1);
            p.pos = axpy(scattering_distance, p.dir, p.pos);
            rayleigh_scatter(p, rng);
            p.history |= CHR_RAYLEIGH_SCATTER;
            p.last_hit = -1;
            return CONTINUE;
        }
    }
    if (use_weights) p.weight *= chr_expf(-s.distance / s.absorption_length);
    p.pos = axpy(s.distance, p.dir, p.pos);
    p.time = p.time + s.distance / (SPEED_OF_LIGHT / s.n1);
    return PASS;
}

// photon.h:572-632 (Fresnel)
__device__ __forceinline__ void propagate_at_boundary(Photon &p, const State &s, chr_xorwow &rng) {
    const float incident_angle = get_theta(s.normal, -p.dir);
    const float refracted_angle = chr_asinf((chr_sinf(incident_angle) * s.n1) / s.n2);
    V3 ipn = cross(p.dir, s.normal);
    const float ipn_len = norm(ipn);
    if (ipn_len < 1e-6f) ipn = p.pol; else ipn = ipn / ipn_len;
    const float nc = dot(p.pol, ipn);
    const float normal_probability = nc * nc;
    float rc;
    if (chr_uniform01(&rng) < normal_probability) {
        rc = -chr_sinf(incident_angle - refracted_angle) / chr_sinf(incident_angle + refracted_angle);
        if ((chr_uniform01(&rng) < rc * rc) || chr_isnan(refracted_angle)) {
            p.dir = rotate(s.normal, incident_angle, ipn);
            p.history |= CHR_REFLECT_SPECULAR;
        } else {
            p.dir = rotate(s.normal, PI_F - refracted_angle, ipn);
        }
        p.pol = ipn;
    } else {
        rc = chr_tanf(incident_angle - refracted_angle) / chr_tanf(incident_angle + refracted_angle);
        if ((chr_uniform01(&rng) < rc * rc) || chr_isnan(refracted_angle)) {
            p.dir = rotate(s.normal, incident_angle, ipn);
            p.history |= CHR_REFLECT_SPECULAR;
        } else {
            p.dir = rotate(s.normal, PI_F - refracted_angle, ipn);
        }
        p.pol = cross(ipn, p.dir);
        p.pol = p.pol / norm(p.pol);
    }
}

// photon.h:634-667
__device__ __forceinline__ int specular_reflector(Photon &p, const State &s) {
    const float incident_angle = get_theta(s.normal, -p.dir);
    V3 ipn = cross(p.dir, s.normal);
    ipn = ipn / norm(ipn);
    p.dir = rotate(s.normal, incident_angle, ipn);
    p.history |= CHR_REFLECT_SPECULAR;
    return CONTINUE;
}

__device__ __forceinline__ int diffuse_reflector(Photon &p, const State &s, chr_xorwow &rng) {
    float ndotv;
    do {
        p.dir = uniform_sphere(rng);
        ndotv = dot(p.dir, s.normal);
        if (ndotv < 0.0f) { p.dir = -p.dir; ndotv = -ndotv; }
    } while (!(chr_uniform01(&rng) < ndotv));
    p.pol = cross(uniform_sphere(rng), p.dir);
    p.pol = p.pol / norm(p.pol);
    p.history |= CHR_REFLECT_DIFFUSE;
    return CONTINUE;
}

// cuComplex semantics (CUDA toolkit cuComplex.h) + cx.h:1-35
struct Cx { float r, i; };
__device__ __forceinline__ Cx cxm(float r, float i) { return Cx{r, i}; }
__device__ __forceinline__ Cx cadd(Cx a, Cx b) { return cxm(a.r + b.r, a.i + b.i); }
__device__ __forceinline__ Cx csub(Cx a, Cx b) { return cxm(a.r - b.r, a.i - b.i); }
__device__ __forceinline__ Cx cmul(Cx a, Cx b) {
    return cxm(__builtin_fmaf(a.r, b.r, -(a.i * b.i)), __builtin_fmaf(a.r, b.i, a.i * b.r));
}
__device__ __forceinline__ Cx cdiv(Cx x, Cx y) {
    float s = chr_fabsf(y.r) + chr_fabsf(y.i);
    float oos = 1.0f / s;
    const float ars = x.r * oos, ais = x.i * oos, brs = y.r * oos, bis = y.i * oos;
    s = __builtin_fmaf(bis, bis, brs * brs);
    oos = 1.0f / s;
    return cxm(__builtin_fmaf(ais, bis, ars * brs) * oos, __builtin_fmaf(ais, brs, -(ars * bis)) * oos);
}
__device__ __forceinline__ float cabs_(Cx x) {
    const float a = chr_fabsf(x.r), b = chr_fabsf(x.i);
    float v, w, t;
    if (a > b) { v = a; w = b; } else { v = b; w = a; }
    t = w / v;
    t = __builtin_fmaf(t, t, 1.0f);
    t = v * chr_sqrtf(t);
    if ((v == 0.0f) || (v > 3.402823466e38f) || (w > 3.402823466e38f)) t = v + w;
    return t;
}
__device__ __forceinline__ float carg_(Cx x) { return chr_atan2f(x.i, x.r); }
__device__ __forceinline__ Cx csqrt_(Cx x) {
    const float r = chr_sqrtf(cabs_(x));
    const float t = carg_(x) / 2.0f;
    float st, ct;
    chr_sincosf(t, &st, &ct);
    return cxm(r * ct, r * st);
}

// photon.h:669-827 (thin film); rare path, kept out of line
__device__ CHR_COLD int propagate_complex(const DevGeom &g, Photon &p, const State &s, chr_xorwow &rng,
                                              const DevSurface &sf, int use_weights) {
    const float *T = g.tables;
    float detect = interp_property(g, p.wavelength, T + sf.detect);
    const float reflect_diffuse = interp_property(g, p.wavelength, T + sf.reflect_diffuse);
    const float n2_eta = interp_property(g, p.wavelength, T + sf.eta);
    const float n2_k = interp_property(g, p.wavelength, T + sf.k);
    const Cx n1 = cxm(s.n1, 0.0f), n2 = cxm(n2_eta, n2_k), n3 = cxm(s.n2, 0.0f);
    float cos_t1 = dot(p.dir, s.normal);
    if (cos_t1 < 0.0f) cos_t1 = -cos_t1;
    const float theta = chr_acosf(cos_t1);
    float sth, cth;
    chr_sincosf(theta, &sth, &cth);
    const Cx cos1 = cxm(cth, 0.0f), sin1 = cxm(sth, 0.0f);
    const float e = ((2.0f * PI_F) * sf.thickness) / p.wavelength;
    const Cx r13 = cdiv(n1, n3), r12 = cdiv(n1, n2);
    const Cx ratio13sin = cmul(cmul(r13, r13), cmul(sin1, sin1));
    const Cx cos3 = csqrt_(csub(cxm(1.0f, 0.0f), ratio13sin));
    const Cx ratio12sin = cmul(cmul(r12, r12), cmul(sin1, sin1));
    const Cx cos2 = csqrt_(csub(cxm(1.0f, 0.0f), ratio12sin));
    const Cx n2c2 = cmul(n2, cos2);
    const float u = n2c2.r, v = n2c2.i;
    const Cx two = cxm(2.0f, 0.0f);
    const Cx s_n1c1 = cmul(n1, cos1), s_n2c2 = cmul(n2, cos2), s_n3c3 = cmul(n3, cos3);
    const Cx s_r12 = cdiv(csub(s_n1c1, s_n2c2), cadd(s_n1c1, s_n2c2));
    const Cx s_r23 = cdiv(csub(s_n2c2, s_n3c3), cadd(s_n2c2, s_n3c3));
    const Cx s_t12 = cdiv(cmul(two, s_n1c1), cadd(s_n1c1, s_n2c2));
    const Cx s_t23 = cdiv(cmul(two, s_n2c2), cadd(s_n2c2, s_n3c3));
    const Cx s_g = cdiv(s_n3c3, s_n1c1);
    const float s_abs_r12 = cabs_(s_r12), s_abs_r23 = cabs_(s_r23), s_abs_t12 = cabs_(s_t12), s_abs_t23 = cabs_(s_t23);
    const float s_arg_r12 = carg_(s_r12), s_arg_r23 = carg_(s_r23);
    const float s_exp1 = chr_expf((2.0f * v) * e);
    const float s_exp2 = 1.0f / s_exp1;
    const float two_ue = (2.0f * u) * e;
    const float s_denom = s_exp1 + ((s_abs_r12 * s_abs_r12) * (s_abs_r23 * s_abs_r23)) * s_exp2 +
                          ((2.0f * s_abs_r12) * s_abs_r23) * chr_cosf(s_arg_r23 + s_arg_r12 + two_ue);
    float s_r = (s_abs_r12 * s_abs_r12) * s_exp1 + (s_abs_r23 * s_abs_r23) * s_exp2 +
                ((2.0f * s_abs_r12) * s_abs_r23) * chr_cosf(s_arg_r23 - s_arg_r12 + two_ue);
    s_r /= s_denom;
    float s_t = ((s_g.r * (s_abs_t12 * s_abs_t12)) * s_abs_t23) * s_abs_t23;
    s_t /= s_denom;
    const Cx p_n2c1 = cmul(n2, cos1), p_n3c2 = cmul(n3, cos2), p_n2c3 = cmul(n2, cos3), p_n1c2 = cmul(n1, cos2);
    const Cx p_r12 = cdiv(csub(p_n2c1, p_n1c2), cadd(p_n2c1, p_n1c2));
    const Cx p_r23 = cdiv(csub(p_n3c2, p_n2c3), cadd(p_n3c2, p_n2c3));
    const Cx p_t12 = cdiv(cmul(cmul(two, n1), cos1), cadd(p_n2c1, p_n1c2));
    const Cx p_t23 = cdiv(cmul(cmul(two, n2), cos2), cadd(p_n3c2, p_n2c3));
    const Cx p_g = cdiv(cmul(n3, cos3), cmul(n1, cos1));
    const float p_abs_r12 = cabs_(p_r12), p_abs_r23 = cabs_(p_r23), p_abs_t12 = cabs_(p_t12), p_abs_t23 = cabs_(p_t23);
    const float p_arg_r12 = carg_(p_r12), p_arg_r23 = carg_(p_r23);
    const float p_exp1 = chr_expf((2.0f * v) * e);
    const float p_exp2 = 1.0f / p_exp1;
    const float p_denom = p_exp1 + ((p_abs_r12 * p_abs_r12) * (p_abs_r23 * p_abs_r23)) * p_exp2 +
                          ((2.0f * p_abs_r12) * p_abs_r23) * chr_cosf(p_arg_r23 + p_arg_r12 + two_ue);
    float p_r = (p_abs_r12 * p_abs_r12) * p_exp1 + (p_abs_r23 * p_abs_r23) * p_exp2 +
                ((2.0f * p_abs_r12) * p_abs_r23) * chr_cosf(p_arg_r23 - p_arg_r12 + two_ue);
    p_r /= p_denom;
    float p_t = ((p_g.r * (p_abs_t12 * p_abs_t12)) * p_abs_t23) * p_abs_t23;
    p_t /= p_denom;
    const float incident_angle = get_theta(s.normal, -p.dir);
    const float refracted_angle = chr_asinf((chr_sinf(incident_angle) * s.n1) / s.n2);
    V3 ipn = cross(p.dir, s.normal);
    const float ipn_len = norm(ipn);
    if (ipn_len < 1e-6f) ipn = p.pol; else ipn = ipn / ipn_len;
    const float nc = dot(p.pol, ipn);
    const float normal_probability = nc * nc;
    float transmit = __builtin_fmaf(normal_probability, s_t, (1.0f - normal_probability) * p_t);
    if (!sf.transmissive) transmit = 0.0f;
    float reflect = __builtin_fmaf(normal_probability, s_r, (1.0f - normal_probability) * p_r);
    float absorb = 1.0f - transmit - reflect;
    if (use_weights && p.weight > WEIGHT_LOWER_THRESHOLD && absorb < (1.0f - WEIGHT_LOWER_THRESHOLD)) {
        const float survive = 1.0f - absorb;
        absorb = 0.0f;
        p.weight *= survive;
        detect /= survive; reflect /= survive; transmit /= survive;
    }
    if (use_weights && detect > 0.0f) {
        p.history |= CHR_SURFACE_DETECT;
        p.weight *= detect;
        return BREAK;
    }
    const float us = chr_uniform01(&rng);
    if (us < absorb) {
        const float usd = chr_uniform01(&rng);
        if (usd < detect) p.history |= CHR_SURFACE_DETECT;
        else p.history |= CHR_SURFACE_ABSORB;
        return BREAK;
    } else if (us < absorb + reflect || !sf.transmissive) {
        const float usr = chr_uniform01(&rng);
        if (usr < reflect_diffuse) return diffuse_reflector(p, s, rng);
        return specular_reflector(p, s);
    }
    p.dir = rotate(s.normal, PI_F - refracted_angle, ipn);
    p.pol = cross(ipn, p.dir);
    p.pol = p.pol / norm(p.pol);
    p.history |= CHR_SURFACE_TRANSMIT;
    return CONTINUE;
}

// photon.h:829-874
__device__ CHR_COLD int propagate_at_wls(const DevGeom &g, Photon &p, const State &s, chr_xorwow &rng,
                                             const DevSurface &sf, int use_weights) {
    const float *T = g.tables;
    float absorb = interp_property(g, p.wavelength, T + sf.absorb);
    float reflect_specular = interp_property(g, p.wavelength, T + sf.reflect_specular);
    float reflect_diffuse = interp_property(g, p.wavelength, T + sf.reflect_diffuse);
    const float reemit = interp_property(g, p.wavelength, T + sf.reemit);
    const float us = chr_uniform01(&rng);
    if (use_weights && p.weight > WEIGHT_LOWER_THRESHOLD && absorb < (1.0f - WEIGHT_LOWER_THRESHOLD)) {
        const float survive = 1.0f - absorb;
        absorb = 0.0f;
        p.weight *= survive;
        reflect_diffuse /= survive;
        reflect_specular /= survive;
    }
    if (us < absorb) {
        const float usr = chr_uniform01(&rng);
        if (usr < reemit) {
            p.history |= CHR_SURFACE_REEMIT;
            p.wavelength = sample_cdf(rng, (int)g.wl_n, g.wl_start, g.wl_step, T + sf.reemission_cdf);
            p.dir = uniform_sphere(rng);
            p.pol = cross(uniform_sphere(rng), p.dir);
            p.pol = p.pol / norm(p.pol);
            return CONTINUE;
        }
        p.history |= CHR_SURFACE_ABSORB;
        return BREAK;
    } else if (us < absorb + reflect_specular + reflect_diffuse) {
        const float usr = chr_uniform01(&rng) * (reflect_specular + reflect_diffuse);
        if (usr < reflect_specular) return specular_reflector(p, s);
        return diffuse_reflector(p, s, rng);
    }
    p.history |= CHR_SURFACE_TRANSMIT;
    return PASS;
}

// photon.h:877-907 (iidx+1 clamped at the last angle, see oracle)
__device__ CHR_COLD int propagate_at_dichroic(const DevGeom &g, Photon &p, const State &s, chr_xorwow &rng,
                                                  const DevSurface &sf) {
    const float *T = g.tables;
    const float incident_angle = get_theta(s.normal, -p.dir);
    const int na = (int)sf.dichroic_nangles;
    const float idx = interp_idx(incident_angle, na, T + sf.dichroic_angles);
    const uint32_t iidx = (uint32_t)(int)idx;
    const uint32_t ihi = (iidx + 1 < (uint32_t)na) ? iidx + 1 : (uint32_t)na - 1;
    const uint32_t W1 = g.wl_n + 1;
    const float rlo = interp_property(g, p.wavelength, T + sf.dichroic_reflect + iidx * W1);
    const float rhi = interp_property(g, p.wavelength, T + sf.dichroic_reflect + ihi * W1);
    const float tlo = interp_property(g, p.wavelength, T + sf.dichroic_transmit + iidx * W1);
    const float thi = interp_property(g, p.wavelength, T + sf.dichroic_transmit + ihi * W1);
    const float fr = idx - (float)iidx;
    const float reflect_prob = __builtin_fmaf(rhi - rlo, fr, rlo);
    const float transmit_prob = __builtin_fmaf(thi - tlo, fr, tlo);
    const float us = chr_uniform01(&rng);
    if (us < reflect_prob) return specular_reflector(p, s);
    if (us < transmit_prob + reflect_prob) { p.history |= CHR_SURFACE_TRANSMIT; return PASS; }
    p.history |= CHR_SURFACE_ABSORB;
    return BREAK;
}

// photon.h:909-951
__device__ CHR_COLD int propagate_at_angular(const DevGeom &g, Photon &p, const State &s, chr_xorwow &rng,
                                                 const DevSurface &sf, int use_weights) {
    const float *T = g.tables;
    const float incident_angle = get_theta(s.normal, -p.dir);
    const int na = (int)sf.angular_nangles;
    const float idx = interp_idx(incident_angle, na, T + sf.angular_angles);
    const uint32_t iidx = (uint32_t)(int)idx;
    const uint32_t ihi = (iidx + 1 < (uint32_t)na) ? iidx + 1 : (uint32_t)na - 1;
    const float t = idx - (float)iidx;
    const float *tr = T + sf.angular_transmit, *rsp = T + sf.angular_reflect_specular, *rdf = T + sf.angular_reflect_diffuse;
    float tp = __builtin_fmaf(t, tr[ihi] - tr[iidx], tr[iidx]);
    float rs = __builtin_fmaf(t, rsp[ihi] - rsp[iidx], rsp[iidx]);
    float rd = __builtin_fmaf(t, rdf[ihi] - rdf[iidx], rdf[iidx]);
    float ap = 1.0f - tp - rs - rd;
    if (use_weights && p.weight > WEIGHT_LOWER_THRESHOLD && ap < (1.0f - WEIGHT_LOWER_THRESHOLD)) {
        const float survive = 1.0f - ap;
        ap = 0.0f;
        p.weight *= survive;
        tp /= survive; rs /= survive; rd /= survive;
    }
    const float us = chr_uniform01(&rng);
    if (us < ap) { p.history |= CHR_SURFACE_ABSORB; return BREAK; }
    if (us < ap + tp) { p.history |= CHR_SURFACE_TRANSMIT; return PASS; }
    if (us < ap + tp + rs) return specular_reflector(p, s);
    return diffuse_reflector(p, s, rng);
}

// photon.h:953-1037
__device__ __forceinline__ int propagate_at_surface(const DevGeom &g, Photon &p, const State &s, chr_xorwow &rng,
                                                    int use_weights) {
    const DevSurface &sf = g.surfaces[s.surface_index];
    if (sf.model == CHR_SURFACE_COMPLEX) return propagate_complex(g, p, s, rng, sf, use_weights);
    if (sf.model == CHR_SURFACE_WLS) return propagate_at_wls(g, p, s, rng, sf, use_weights);
    if (sf.model == CHR_SURFACE_DICHROIC) return propagate_at_dichroic(g, p, s, rng, sf);
    if (sf.model == CHR_SURFACE_ANGULAR) return propagate_at_angular(g, p, s, rng, sf, use_weights);
    const float *T = g.tables;
    float detect = interp_property(g, p.wavelength, T + sf.detect);
    float absorb = interp_property(g, p.wavelength, T + sf.absorb);
    float reflect_diffuse = interp_property(g, p.wavelength, T + sf.reflect_diffuse);
    float reflect_specular = interp_property(g, p.wavelength, T + sf.reflect_specular);
    const float us = chr_uniform01(&rng);
    if (use_weights && p.weight > WEIGHT_LOWER_THRESHOLD && absorb < (1.0f - WEIGHT_LOWER_THRESHOLD)) {
        const float survive = 1.0f - absorb;
        absorb = 0.0f;
        p.weight *= survive;
        detect /= survive; reflect_diffuse /= survive; reflect_specular /= survive;
    }
    if (use_weights && detect > 0.0f) {
        p.history |= CHR_SURFACE_DETECT;
        p.weight *= detect;
        return BREAK;
    }
    if (us < absorb) { p.history |= CHR_SURFACE_ABSORB; return BREAK; }
    if (us < absorb + detect) { p.history |= CHR_SURFACE_DETECT; return BREAK; }
    if (us < absorb + detect + reflect_diffuse) return diffuse_reflector(p, s, rng);
    if (us < absorb + detect + reflect_diffuse + reflect_specular) return specular_reflector(p, s);
    return PASS;
}

// ---------------------------------------------------------------- kernels
struct PropagateArgs {
    float *pos, *dir, *pol, *wl, *t, *weights;
    uint32_t *flags;
    int32_t *last_hit;
    uint32_t *evidx;
    uint32_t *rng;
    uint32_t nslots;
    const uint32_t *input_queue;
    int32_t first, nthreads, max_steps, use_weights, scatter_first;
    unsigned long long *alive_masks;   // one word per 64 slots
    uint32_t *counters;                // [0]: stack overflows
    const uint32_t *order;             // coherence order: work-item t runs slot order[t] (nullptr: t)
    const int2 *hits;                  // shade_kernel: walk result per queue position (trace_kernel)
    uint32_t *diag;                    // multi-step kernels (nullptr: off): [0] += flat walks walked whole,
                                       // [1] max steps of one photon, [2..3] u64 max of (cycles << 16 | steps),
                                       // [4..13] u64 sums over photons of > 64 steps (tail kernel): walk
                                       // ticks, step ticks, walk iterations, steps, photons
    // device-driven steps (nullptr: host-driven): the queue length is *dev_n - 1
    // and the launch runs only if *mode == want
    const uint32_t *dev_n;
    const uint32_t *mode;
    uint32_t prio;                     // tail kernel: raise its waves' issue priority (s_setprio; the
                                       // batches' tail, the critical path beside the next batch's walk)
    uint32_t pair;                     // tail kernel: a lone walk takes an idle wave of its workgroup as
                                       // triangle tester (walk_pair; CHR_PAIR_WALK=0: walk_lone alone)
    uint32_t walk_up;                  // tail kernel: a walk with a previous hit starts at that hit's leaf
                                       // and climbs (CHR_WALK_UP: 0 none, 1 lone and grouped, 2 lone only,
                                       // 4 as 1 without the chain prefetch)
    uint32_t want;
    // tail kernel, work-queue mode (nullptr: group g runs queue positions g, g + cap, ...): a
    // zeroed counter the photon groups take queue positions from, for queues no longer than
    // the slot count (each position then its own RNG slot, loaded and stored per photon)
    uint32_t *work;
};
// modes of a device-driven step slot (step_head_kernel)
constexpr uint32_t STEP_IDLE = 0, STEP_ONE = 1, STEP_TAIL = 2;

__device__ __forceinline__ V3 load3(const float *p, uint32_t i) { return v3(p[3 * i], p[3 * i + 1], p[3 * i + 2]); }
__device__ __forceinline__ void store3(float *p, uint32_t i, V3 v) { p[3 * i] = v.x; p[3 * i + 1] = v.y; p[3 * i + 2] = v.z; }

// One live photon through the step loop of propagate.cu:279-341 (the caller
// has checked the entry history against DEAD_MASK, propagate.cu:283-284) and
// its write-back (propagate.cu:343-353).  Returns whether it is still alive.
template <int BATCH, int WIDE, bool COUNT>
__device__ __forceinline__ bool run_photon(const DevGeom &g, const PropagateArgs &a, uint32_t photon_id,
                                           uint32_t history, chr_xorwow &rng, Stack st, WStack &wst,
                                           uint32_t &overflow, WalkCounts &cnt, int *steps_run = nullptr) {
    Photon p;
    p.history = history;
    p.pos = load3(a.pos, photon_id);
    p.dir = load3(a.dir, photon_id);
    p.dir = p.dir / norm(p.dir);
    p.pol = load3(a.pol, photon_id);
    p.pol = p.pol / norm(p.pol);
    p.wavelength = a.wl[photon_id];
    p.time = a.t[photon_id];
    p.last_hit = a.last_hit[photon_id];
    p.weight = a.weights[photon_id];
    State s;
    int scatter_first = a.scatter_first;
    int steps = 0;
    unsigned long long tstart = 0;
    if constexpr (COUNT) tstart = __builtin_amdgcn_s_memtime();
    while (steps < a.max_steps) {
        steps++;
        const float prod = ((((p.dir.x * p.dir.y) * p.dir.z) * p.pos.x) * p.pos.y) * p.pos.z;
        if (chr_isnan(prod)) { p.history |= CHR_NO_HIT | CHR_NAN_ABORT; break; }
        unsigned long long t0 = 0;
        if constexpr (COUNT) t0 = __builtin_amdgcn_s_memtime();
        fill_state<BATCH, WIDE, COUNT>(g, s, p, st, wst, overflow, cnt);
        if constexpr (COUNT) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            if (wave_leader()) cnt.wave_fill_cycles += t1 - t0;
        }
        if (p.last_hit == -1) break;
        int command = propagate_to_boundary(g, p, s, rng, a.use_weights, scatter_first);
        scatter_first = 0;
        if (command == BREAK) break;
        if (command == CONTINUE) continue;
        if (s.surface_index != -1) {
            command = propagate_at_surface(g, p, s, rng, a.use_weights);
            if (command == BREAK) break;
            if (command == CONTINUE) continue;
        }
        propagate_at_boundary(p, s, rng);
    }
    if constexpr (COUNT) {
        const unsigned long long tend = __builtin_amdgcn_s_memtime();
        if (wave_leader()) cnt.wave_other_cycles += tend - tstart;   // includes fill; split on the host
    }
    if (steps_run) *steps_run = steps;
    store3(a.pos, photon_id, p.pos);
    store3(a.dir, photon_id, p.dir);
    store3(a.pol, photon_id, p.pol);
    a.wl[photon_id] = p.wavelength;
    a.t[photon_id] = p.time;
    a.flags[photon_id] = p.history;
    a.last_hit[photon_id] = p.last_hit;
    a.weights[photon_id] = p.weight;
    return (p.history & DEAD_MASK) == 0;
}

__device__ __forceinline__ void load_rng(const PropagateArgs &a, uint32_t slot, chr_xorwow &rng) {
    const uint32_t ns = a.nslots;
    rng.d = a.rng[slot]; rng.v0 = a.rng[ns + slot]; rng.v1 = a.rng[2 * ns + slot];
    rng.v2 = a.rng[3 * ns + slot]; rng.v3 = a.rng[4 * ns + slot]; rng.v4 = a.rng[5 * ns + slot];
}
__device__ __forceinline__ void store_rng(const PropagateArgs &a, uint32_t slot, const chr_xorwow &rng) {
    const uint32_t ns = a.nslots;
    a.rng[slot] = rng.d; a.rng[ns + slot] = rng.v0; a.rng[2 * ns + slot] = rng.v1;
    a.rng[3 * ns + slot] = rng.v2; a.rng[4 * ns + slot] = rng.v3; a.rng[5 * ns + slot] = rng.v4;
}

template <bool COUNT>
__device__ __forceinline__ void flush_counters(const PropagateArgs &a, uint32_t overflow, const WalkCounts &cnt) {
    if (overflow) atomicAdd(a.counters, overflow);
    if constexpr (COUNT) {
        unsigned long long *c64 = reinterpret_cast<unsigned long long *>(a.counters + 2);
        atomicAdd(c64, (unsigned long long)cnt.nodes);
        atomicAdd(c64 + 1, (unsigned long long)cnt.tris);
        atomicAdd(c64 + 2, (unsigned long long)cnt.walks);
        atomicAdd(c64 + 3, (unsigned long long)cnt.wave_nodes);
        atomicAdd(c64 + 4, (unsigned long long)cnt.wave_tris);
        atomicAdd(c64 + 5, cnt.wave_fill_cycles);
        atomicAdd(c64 + 6, cnt.wave_other_cycles);
    }
}

// propagate.cu:254-366, one chunk per launch (the reference's launch
// structure; used when the slot count is not a multiple of 64).
// BATCH: children fetched together per group (exact-order walk);
// MINW: minimum waves per SIMD requested from the register allocator.
// WIDE: 0 exact-order walk of the reference BVH, 1 wide BVH node loop,
// 1000 + b: wide BVH scheduled walk, triangle batch threshold b (0: per-lane choice).
template <int BATCH, int MINW, int WIDE, bool COUNT = false>
__global__ __launch_bounds__(BLOCK, MINW) void propagate_kernel(const DevGeom *__restrict__ gdev, PropagateArgs a) {
    __shared__ uint32_t lds_stack[WIDE ? lds_words(WIDE) * BLOCK : STACK_LDS * BLOCK];
    const int tid = blockIdx.x * BLOCK + threadIdx.x;
    unsigned alive = 0;
    // A photon's RNG slot and queue position are its slot id, whichever
    // work-item runs it: the coherence order only changes which rays share a
    // wave, never what any photon computes.
    const int id = (a.order && tid < a.nthreads) ? (int)a.order[tid] : tid;
    if (tid < a.nthreads) {
        const uint32_t photon_id = a.input_queue[a.first + id];
        const uint32_t history = a.flags[photon_id] & 0xFFFFu;   // unsigned short on the device (photon.h:29)
        if (!(history & DEAD_MASK)) {
            chr_xorwow rng;
            load_rng(a, (uint32_t)id, rng);
            Stack st;
            WStack wst;
            st.lds = (CHR_LDS uint32_t *)(lds_stack + threadIdx.x);
            uint2 wspill[WIDE_STACK - WIDE_LDS];
            wst.spill = wspill;
            wst.sstride = 1;
            wst.node = (CHR_LDS uint32_t *)(lds_stack + threadIdx.x);
            wst.dist = (CHR_LDS float *)(lds_stack + WIDE_LDS * BLOCK + threadIdx.x);
    wst.leafq = (CHR_LDS uint32_t *)(lds_stack + 2 * WIDE_LDS * BLOCK + threadIdx.x);
            wst.leafq = (CHR_LDS uint32_t *)(lds_stack + 2 * WIDE_LDS * BLOCK + threadIdx.x);
            uint32_t overflow = 0;
            WalkCounts cnt{0u, 0u, 0u, 0u, 0u, 0ull, 0ull, 0u};
            const DevGeom &g = *gdev;   // device-resident: uniform s_loads, no private copy
            alive = run_photon<BATCH, WIDE, COUNT>(g, a, photon_id, history, rng, st, wst, overflow, cnt);
            store_rng(a, (uint32_t)id, rng);
            flush_counters<COUNT>(a, overflow, cnt);
        }
    }
    if (a.order) {   // masks zeroed by the host; bit per slot
        if (alive) atomicOr(a.alive_masks + (id >> 6), 1ull << (id & 63));
        return;
    }
    const unsigned long long mask = __ballot(alive);
    if ((threadIdx.x & 63) == 0 && id < a.nthreads) a.alive_masks[id >> 6] = mask;
}

// One whole host step in ONE launch (default).  The reference launches the
// queue in chunks of cap = nthreads_per_block*max_blocks photons, one after
// the other, and the photon at queue position q uses RNG slot q mod cap
// (photon.py:266-276, chunk_iterator).  Here work-item `slot` runs queue
// positions slot, slot+cap, slot+2cap, ... in that order with the slot's RNG
// state held in registers: the same photons meet the same states in the same
// order as in the chunked launches, so every result is identical -- but there
// is one launch (and one grid drain) per step instead of ceil(n/cap), and each
// lane's work is a sum over ~n/cap photons, which evens out the lanes of a wave.
// Alive bits are per queue position (a.alive_masks[q >> 6]); requires
// cap % 64 == 0 so that a wave's 64 positions share one mask word.
template <int BATCH, int MINW, int WIDE, bool COUNT = false>
__global__ __launch_bounds__(BLOCK, MINW) void propagate_step_kernel(const DevGeom *__restrict__ gdev,
                                                                     PropagateArgs a, uint32_t cap) {
    __shared__ uint32_t lds_stack[WIDE ? lds_words(WIDE) * BLOCK : STACK_LDS * BLOCK];
    const uint32_t slot = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t n = (uint32_t)a.nthreads;   // queue length of this step
    // whole waves only (cap % 64 == 0); the partial last wave of a short queue
    // stays to write its mask word
    if (slot >= cap || (slot & ~63u) >= n) return;
    Stack st;
    WStack wst;
    st.lds = (CHR_LDS uint32_t *)(lds_stack + threadIdx.x);
    uint2 wspill[WIDE_STACK - WIDE_LDS];
    wst.spill = wspill;
    wst.sstride = 1;
    wst.node = (CHR_LDS uint32_t *)(lds_stack + threadIdx.x);
    wst.dist = (CHR_LDS float *)(lds_stack + WIDE_LDS * BLOCK + threadIdx.x);
    wst.leafq = (CHR_LDS uint32_t *)(lds_stack + 2 * WIDE_LDS * BLOCK + threadIdx.x);
    uint32_t overflow = 0;
    WalkCounts cnt{0u, 0u, 0u, 0u, 0u, 0ull, 0ull, 0u};
    const DevGeom &g = *gdev;
    chr_xorwow rng;
    bool have_rng = false;
    for (uint32_t q = slot & ~63u; q < n; q += cap) {   // wave-uniform trip count
        const uint32_t pos = q + (slot & 63u);
        bool alive = false;
        if (pos < n) {
            const uint32_t photon_id = a.input_queue[pos];
            const uint32_t history = a.flags[photon_id] & 0xFFFFu;   // photon.h:29
            if (!(history & DEAD_MASK)) {
                if (!have_rng) { load_rng(a, slot, rng); have_rng = true; }
                alive = run_photon<BATCH, WIDE, COUNT>(g, a, photon_id, history, rng, st, wst, overflow, cnt);
            }
        }
        const unsigned long long mask = __ballot(alive);
        if ((slot & 63u) == 0) a.alive_masks[q >> 6] = mask;
    }
    if (have_rng) store_rng(a, slot, rng);
    flush_counters<COUNT>(a, overflow, cnt);
}

// Shade pass of a split one-step launch (max_steps == 1): the loop body of
// propagate.cu:286-341 run once per queued photon with the walk result of
// trace_kernel, the photon write-back of 343-353 and the alive mask word per
// 64 queue positions.  A slot's photons (queue positions slot, slot + cap, ...)
// share only the RNG state, so the next photon's queue entry, state and walk
// result are loaded while the current one's physics runs.
// LDS copy of the physics tables (DevGeom::phys: property tables, material and
// surface records) for the kernels that run the step physics: fill_state's and
// the surface models' table reads then cost an LDS round trip instead of a
// dependent L2 one.  All threads of the workgroup call it; returns the geometry
// to use -- tables / materials / surfaces pointing into LDS when they fit in
// cap_words, else g unchanged.
constexpr uint32_t SHADE_PHYS_WORDS = 12288;   // 48 KB: 3 workgroups of shade_kernel<3> per CU
// (only DevGeom::phys_hot_words are copied: the re-emission time CDFs stay in HBM)
constexpr uint32_t TAIL_PHYS_WORDS = 8192;     // 32 KB: 2 tail workgroups (+ 40 KB of walk stacks each)
// The copy is the launch's dynamic LDS, sized to the geometry's hot words (the
// demo and 29k detectors: a few KB of their 32 / 48 KB caps), so a workgroup holds
// only the LDS its geometry needs: host and kernel apply the same rule.
#ifdef CHR_STATIC_PHYS_LDS   // (build-time A/B: the round-5 static arrays at the caps)
__host__ __device__ __forceinline__ uint32_t phys_lds_bytes(const DevGeom &, uint32_t) { return 0u; }
#define CHR_PHYS_LDS(name, cap) __shared__ uint4 name[(cap) / 4]
#else
__host__ __device__ __forceinline__ uint32_t phys_lds_bytes(const DevGeom &g, uint32_t cap_words) {
    return g.phys && g.phys_hot_words <= cap_words ? g.phys_hot_words * 4u : 0u;
}
#define CHR_PHYS_LDS(name, cap) extern __shared__ uint4 name[]
#endif
__device__ __forceinline__ DevGeom phys_cache(const DevGeom &g, uint4 *lds, uint32_t cap_words) {
    DevGeom gl = g;
    if (g.phys && g.phys_hot_words <= cap_words) {   // workgroup-uniform
        // the hot part: tables and records; the time CDFs stay global (tables_g)
        const uint4 *src = reinterpret_cast<const uint4 *>(g.phys);
        for (uint32_t i = threadIdx.x; i < g.phys_hot_words / 4u; i += BLOCK) lds[i] = src[i];
        __syncthreads();
        const uint32_t *base = reinterpret_cast<const uint32_t *>(lds);
        gl.tables = reinterpret_cast<const float *>(base);
        gl.materials = reinterpret_cast<const DevMaterial *>(base + g.mat_off);
        gl.surfaces = reinterpret_cast<const DevSurface *>(base + g.surf_off);
    }
    return gl;
}

struct QueuedPhoton {
    uint32_t pid, history;
    V3 pos, dir, pol;
    float wavelength, time, weight;
    int last_hit;
    int2 hit;
};
// the photon at queue position q; pid: its queue entry when already loaded (the
// shade kernel's two-ahead prefetch), else read here first (a dependent load)
// (KNOWN: pid is the queue entry, no fallback load -- no branch holding a load)
template <bool KNOWN = false>
__device__ __forceinline__ void fetch_queued(const PropagateArgs &a, uint32_t q, QueuedPhoton &f,
                                             uint32_t pid = 0xFFFFFFFFu) {
    f.pid = (KNOWN || pid != 0xFFFFFFFFu) ? pid : a.input_queue[q];
    f.history = a.flags[f.pid] & 0xFFFFu;   // photon.h:29
    f.pos = load3(a.pos, f.pid);
    f.dir = load3(a.dir, f.pid);
    f.pol = load3(a.pol, f.pid);
    f.wavelength = a.wl[f.pid];
    f.time = a.t[f.pid];
    f.weight = a.weights[f.pid];
    f.last_hit = a.last_hit[f.pid];
    f.hit = a.hits[q];
}
// The queue entry of the photon two positions ahead is loaded one iteration
// early, so the next photon's state loads go out without first waiting for its
// queue entry (a dependent round trip per photon otherwise; r04 ab5: 487.8-488.2 ->
// 489.4 M/s).
// No wait for the write-back (r04 ab9/ab10).  On gfx9 stores count in vmcnt with the loads,
// in issue order, and the compiler waits for a prefetched value with the count of
// the path into its use with the fewest younger operations.  With the prefetch under
// `if (pos + cap < n)` the loop's back edge copied the prefetched photon after this
// iteration's stores with `s_waitcnt vmcnt(0)` (the entry path from the prologue and
// the queue entry's fallback load also leave paths with none younger), so every
// iteration waited for its own stores to be acknowledged.  Here every lane issues the prefetch (position clamped into the queue), the queue entry two
// ahead is always the one loaded (no fallback load), and the first iteration is
// peeled, so every path into the loop has the write-back behind the prefetch: the
// prefetch is waited for at the physics' join, before the stores, and nothing waits
// for the stores.
template <int MINW, bool WIRES = true>
__global__ __launch_bounds__(BLOCK, MINW) void shade_kernel(const DevGeom *__restrict__ gdev, PropagateArgs a,
                                                            uint32_t cap) {
    if (a.mode && *a.mode != a.want) return;
    CHR_PHYS_LDS(phys_lds, SHADE_PHYS_WORDS);   // phys_lds_bytes(SHADE_PHYS_WORDS) of dynamic LDS
    const DevGeom g = phys_cache(*gdev, phys_lds, SHADE_PHYS_WORDS);
    const uint32_t slot = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t n = a.dev_n ? *a.dev_n - 1u : (uint32_t)a.nthreads;
    if (slot >= cap || (slot & ~63u) >= n) return;   // whole waves (cap % 64 == 0)
    chr_xorwow rng;
    bool have_rng = false;
    enum { P_FILL, P_PHYS, P_OTHER };
    Prof<3> pf;
    pf.start(P_OTHER);
    auto clampq = [n](uint32_t q) { return q < n ? q : n - 1u; };
    QueuedPhoton nx;
    fetch_queued(a, clampq(slot), nx);
    uint32_t pid2 = a.input_queue[clampq(slot + cap)];   // queue entry of position pos + cap
    uint32_t pos = slot;
    auto body = [&](uint32_t qb) __attribute__((always_inline)) {
        const QueuedPhoton cur = nx;
        fetch_queued<true>(a, clampq(pos + cap), nx, pid2);
        pid2 = a.input_queue[clampq(pos + 2 * cap)];
        bool alive = false;
        const bool valid = pos < n && !(cur.history & DEAD_MASK);
        Photon p;
        if (valid) {
            if (!have_rng) { load_rng(a, slot, rng); have_rng = true; }
            p.history = cur.history;
            p.pos = cur.pos;
            p.dir = cur.dir / norm(cur.dir);
            p.pol = cur.pol / norm(cur.pol);
            p.wavelength = cur.wavelength;
            p.time = cur.time;
            p.last_hit = cur.last_hit;
            p.weight = cur.weight;
            const float prod = ((((p.dir.x * p.dir.y) * p.dir.z) * p.pos.x) * p.pos.y) * p.pos.z;
            if (chr_isnan(prod)) {
                p.history |= CHR_NO_HIT | CHR_NAN_ABORT;
            } else {
                State s;
                const int tri = cur.hit.x;
                s.distance = __int_as_float(cur.hit.y);
                pf.tick(P_FILL);
                pf.call(P_FILL);
                Watch wt;
                wt.begin(1u, cur.pid, a.pos, pos, slot, p.pos, p.dir, p.last_hit);
                finish_fill<true, WIRES>(g, s, p, tri);
                wt.filled(tri, s);
                pf.tick(P_PHYS);
                if (p.last_hit != -1) {
                    pf.call(P_PHYS);
                    int command = propagate_to_boundary(g, p, s, rng, a.use_weights, a.scatter_first);
                    if (command == PASS && s.surface_index != -1)
                        command = propagate_at_surface(g, p, s, rng, a.use_weights);
                    if (command == PASS) propagate_at_boundary(p, s, rng);
                }
                wt.end(p.pos, p.history, p.time);
                pf.tick(P_OTHER);
            }
            alive = (p.history & DEAD_MASK) == 0;
        }
        // the prefetched photon and queue entry waited for here, on every path and
        // before the write-back (see above)
        asm volatile("" ::"v"(nx.pid), "v"(nx.history), "v"(nx.pos.x), "v"(nx.pos.y), "v"(nx.pos.z), "v"(nx.dir.x),
                     "v"(nx.dir.y), "v"(nx.dir.z), "v"(nx.pol.x), "v"(nx.pol.y), "v"(nx.pol.z));
        asm volatile("" ::"v"(nx.wavelength), "v"(nx.time), "v"(nx.weight), "v"(nx.last_hit), "v"(nx.hit.x),
                     "v"(nx.hit.y), "v"(pid2));
        if (valid) {
            const uint32_t pid = cur.pid;
            store3(a.pos, pid, p.pos);
            store3(a.dir, pid, p.dir);
            store3(a.pol, pid, p.pol);
            a.wl[pid] = p.wavelength;
            a.t[pid] = p.time;
            a.flags[pid] = p.history;
            a.last_hit[pid] = p.last_hit;
            a.weights[pid] = p.weight;
        }
        const unsigned long long mask = __ballot(alive);
        if ((slot & 63u) == 0) a.alive_masks[qb >> 6] = mask;
    };
    uint32_t qb = slot & ~63u;                         // wave-uniform trip count
    if (qb < n) {
        // the first iteration peeled: the loop's first wait for the prefetched queue
        // entry and state then has this iteration's write-back behind it on every
        // path into the loop (from the prologue it would be the youngest load: vmcnt(0))
        body(qb);
        qb += cap;
        pos += cap;
    }
    for (; qb < n; qb += cap, pos += cap) body(qb);
    if (have_rng) store_rng(a, slot, rng);
#ifdef CHR_DEVICE_PROFILE
    pf.tick(P_OTHER);
    prof_add(CHR_PROF_FILL_MATERIAL, pf.calls[P_FILL], pf.cyc[P_FILL]);
    prof_add(CHR_PROF_SHADE_PHYSICS, pf.calls[P_PHYS], pf.cyc[P_PHYS]);
    prof_add(CHR_PROF_SHADE_OTHER, 0ull, pf.cyc[P_OTHER]);
    prof_add(CHR_PROF_SHADE_KERNEL, 1ull, pf.total());
#endif
}


// ---------------------------------------------------------------- wave-adaptive tail
// The multi-step tail launch lasts as long as its longest-lived photon: on the
// 29k detector one photon bouncing ~500 times between opposite walls set
// 12-25 ms launches at ~25 us per step (r02 tail diagnostics), with the rest of
// the chip idle.  Here the 64 lanes of a wave hold 8 photons (8 lanes each, as
// propagate_group_kernel) and run one step of each per iteration; the walk of
// an iteration spreads the whole wave over the photons that walk in it: with w
// walkers each gets a segment of Gs = 64 / pow2ceil(w) lanes = P = Gs/8
// sub-groups of 8, and a segment advances P depth-first cursors over one
// shared LDS stack (P nodes per dependent fetch), then tests every triangle of
// the iteration's hit leaves at once, one per lane (not leaf after leaf).  The
// physics of a step stays with the photon's own 8 lanes.  Culling uses the
// segment's best of the previous iteration (never below the final one) and the
// nearest hit is the min over (distance, reference rank) with the reference
// leaf check of every other walk, so the result does not depend on P.
constexpr int TAIL_STACK = 128;   // stack entries per 8 lanes; a segment of Gs lanes holds TAIL_STACK * Gs / 8
constexpr int TAIL_TRI = 4 * 64;  // triangle-list words per wave and buffer (<= 4 triangles per lane per iteration)

// 64-bit min over the 8 lanes of each aligned lane group, by DPP (quad xor 1,
// quad xor 2, half-row mirror): VALU moves, no LDS round trips.
__device__ __forceinline__ unsigned long long dpp_min8(unsigned long long k) {
    auto step = [](unsigned long long v, auto ctrl) {
        const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)v, decltype(ctrl)::value, 0xF, 0xF, true);
        const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), decltype(ctrl)::value, 0xF, 0xF, true);
        const unsigned long long o = ((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo;
        return o < v ? o : v;
    };
    k = step(k, std::integral_constant<int, 0xB1>());    // quad_perm [1,0,3,2]
    k = step(k, std::integral_constant<int, 0x4E>());    // quad_perm [2,3,0,1]
    k = step(k, std::integral_constant<int, 0x141>());   // row_half_mirror
    return k;
}

// index of the r-th set bit of m (r < popcount(m))
__device__ __forceinline__ int nth_bit(unsigned long long m, int r) {
    for (int i = 0; i < r; ++i) m &= m - 1;
    return __ffsll((long long)m) - 1;
}

// LDS word arrays of walk_segment: contiguous (the tail kernel's per-wave
// stacks), or a wave's rows of trace_kernel's lane-strided LDS (row r = the 64
// words of the wave's lanes at r * BLOCK), reused when the wave drains.
struct LdsFlat {
    CHR_LDS uint32_t *p;
    __device__ __forceinline__ CHR_LDS uint32_t &operator[](int i) const { return p[i]; }
};
template <int TB>
struct LdsRowsT {
    CHR_LDS uint32_t *p;   // the wave's word 0 (row 0, its first lane)
    int off;
    __device__ __forceinline__ CHR_LDS uint32_t &operator[](int i) const {
        return p[((i + off) >> 6) * TB + ((i + off) & 63)];
    }
};
typedef LdsRowsT<BLOCK> LdsRows;

// Where the lone walker's iteration goes (walk_segment<64>, the tail's
// long-lived photon; device profile build only): wave-cycles of its stack
// refill, its fetch (the loads issued and waited for at once, so the expansion
// after it is compute only), the children's slab tests + near child + pushes +
// triangle list, and the triangle tests + hit reduction; calls = iterations.
template <bool ON>
struct LoneProf {
    __device__ __forceinline__ void begin() {}
    __device__ __forceinline__ void tick(int) {}
    __device__ __forceinline__ void wait_loads() {}
    __device__ __forceinline__ void flush() {}
};
#ifdef CHR_DEVICE_PROFILE
template <>
struct LoneProf<true> {
    unsigned long long cyc[4] = {0ull, 0ull, 0ull, 0ull}, iters = 0ull, t = 0ull;
    __device__ __forceinline__ void begin() { t = __builtin_amdgcn_s_memtime(); iters++; }
    __device__ __forceinline__ void tick(int i) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        cyc[i] += now - t;
        t = now;
    }
    __device__ __forceinline__ void wait_loads() { __builtin_amdgcn_s_waitcnt(0); }
    __device__ __forceinline__ void flush() {
        if (__lane_id() == 0) {
            for (int i = 0; i < 4; ++i) atomicAdd(&chr_prof_cycles[CHR_PROF_LONE_REFILL + i], cyc[i]);
            atomicAdd(&chr_prof_calls[CHR_PROF_LONE_WALK], iters);
            atomicAdd(&chr_prof_cycles[CHR_PROF_LONE_WALK], cyc[0] + cyc[1] + cyc[2] + cyc[3]);
        }
    }
};
#endif

// All 64 lanes call this (converged).  act: the segment has a ray (segment-
// uniform).  Returns the nearest triangle (-1: none) and its distance in
// every lane of the segment.  One dependent global fetch per iteration: the
// triangles of the leaves found in iteration i are fetched together with the
// nodes of iteration i + 1 (their best then culls one iteration later, still
// with a best that never drops below the final one).  best / best_rank /
// best_id seed the walk with a hit already found (a trace_kernel walk handed
// over mid-way): culling with it is conservative, and the result is the min
// over the seed and every triangle this walk tests.
// GS > 0: the segment width as a compile-time constant (GS = 64: one walk on
// the whole wave, the tail's lone long-lived photon -- segment masks and
// offsets fold away); GS = 0: the width Gs_in at run time.
template <int GS, class M, bool UP = false>
__device__ __forceinline__ int walk_segment(const DevGeom &g, bool act, V3 o, V3 d, uint32_t last, int Gs_in, M stk, int cap, M tlist,
                            const TopNodes &top, uint32_t &overflow, float &min_distance, uint32_t &iters,
                            float best = __builtin_inff(), uint32_t best_rank = 0xFFFFFFFFu, int best_id = -1,
                            float best_bd = __builtin_inff(), uint32_t start = 0u) {
    const int Gs = GS ? GS : Gs_in;
    constexpr uint32_t INVALID = 0xFFFFFFFFu;
    constexpr unsigned long long NONE = ~0ull;
    // GS = 64: one ray for the whole wave -- the ray, its best hit and the loop
    // state are wave-uniform; saying so (readfirstlane) lets them live in SGPRs
    // and the loop branch on scalar conditions instead of exec masks
    auto ufl = [](float x) { return GS == 64 ? __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))) : x; };
    auto uu = [](uint32_t x) { return GS == 64 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)x) : x; };
    if (GS == 64) {
        act = uu(act ? 1u : 0u) != 0u;
        o = v3(ufl(o.x), ufl(o.y), ufl(o.z));
        d = v3(ufl(d.x), ufl(d.y), ufl(d.z));
        last = uu(last);
        best = ufl(best);
        best_rank = uu(best_rank);
        best_id = (int)uu((uint32_t)best_id);
        best_bd = ufl(best_bd);
    }
    float cut = ufl(ref_cut(best, best_bd));   // the culling threshold (ref_cut)
    const uint32_t lane = __lane_id();
    const uint32_t seg0 = lane & ~(uint32_t)(Gs - 1);
    const uint32_t L = lane - seg0;                   // lane within the segment
    const uint32_t k = L & 7u;                        // child slot of this lane
    const unsigned long long segmask = Gs == 64 ? ~0ull : (((1ull << Gs) - 1ull) << seg0);
    const unsigned long long below = (1ull << lane) - 1ull;
    const V3 noid = v3(-o.x / d.x, -o.y / d.y, -o.z / d.z);
    const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const RaySlab r = make_slab(o, noid, inv);
    // cursor 0 starts at the root (UP: at start, walk_lone<true>'s climb; per segment)
    uint32_t cur = (act && L < 8u) ? (UP ? start : 0u) : INVALID;
    uint32_t chainw = INVALID;                        // UP: ancestor word k of the cursor's node (lane k)
    float cur_t = 0.0f;
    int sp = 0;
    uint32_t Tp = 0;                                  // triangles listed by the previous iteration
    int pb = 0;                                       // their list buffer (double-buffered)
    bool done = !act;
    iters = 0;
    LoneProf<GS == 64> lp;
    // GS = 64: the loop state (done, the stack depth, the listed triangles) is
    // wave-uniform, said explicitly (uu) so the loop branches on scalars instead of
    // exec masks
    while (true) {
        if constexpr (GS == 64) {
            if (done) break;
        } else {
            if (__ballot(!done) == 0) break;
            if (done) continue;
        }
        iters++;
        lp.begin();
        // cursors without a node take the topmost unculled stack entries: a
        // window of up to 8 entries read at once, the r-th empty cursor (in
        // sub-group order) taking the r-th unculled entry (from the top)
        unsigned long long em = __ballot(k == 0u && cur == INVALID) & segmask;
        const uint32_t lead = lane & ~7u;                 // my sub-group's leader lane
        const bool refill = em != 0 && sp > 0;
        while (em != 0 && sp > 0) {
            const int W = sp < 8 ? sp : 8;
            uint32_t en = 0, et = 0;
            bool ok = false;
            if (L < (uint32_t)W) {
                en = stk[2 * (sp - 1 - (int)L)];
                et = stk[2 * (sp - 1 - (int)L) + 1];
                ok = !(__uint_as_float(et) > cut);            // mesh.h:94-96
            }
            const unsigned long long okm = __ballot(ok) & segmask;
            const int need = __popcll(em), nv = __popcll(okm);
            const int take = need < nv ? need : nv;
            // window lane L's rank among the unculled entries (from the top); the
            // first unculled entry not taken bounds what is consumed (all above it)
            const int rho = __popcll(okm & below);
            const unsigned long long stopm = __ballot(ok && rho == take) & segmask;
            const int consumed = stopm ? (__ffsll((long long)stopm) - 1 - (int)seg0) : W;
            // the r-th empty cursor takes the r-th unculled entry, through the
            // segment's free triangle-list buffer (written two iterations ago,
            // tested one ago): no per-lane bit searches
            if (ok && rho < take) {
                tlist[(pb ^ 1) * TAIL_TRI + 2 * rho] = en;
                tlist[(pb ^ 1) * TAIL_TRI + 2 * rho + 1] = et;
            }
            __builtin_amdgcn_wave_barrier();
            // GS = 64: all 8 lanes of an empty cursor's sub-group read the entry it
            // takes (an LDS broadcast), no shuffle from the leader follows; otherwise
            // the leader takes it and its sub-group reads it by shuffle below
            const bool empty = GS == 64 ? ((em >> lead) & 1ull) != 0 : (k == 0u && cur == INVALID);
            const int rnk = __popcll(em & (GS == 64 ? ((1ull << lead) - 1ull) : below));
            const unsigned long long taken = __ballot(k == 0u && empty && rnk < take) & segmask;
            if (empty && rnk < take) {
                cur = tlist[(pb ^ 1) * TAIL_TRI + 2 * rnk];
                cur_t = __uint_as_float(tlist[(pb ^ 1) * TAIL_TRI + 2 * rnk + 1]);
            }
            __builtin_amdgcn_wave_barrier();
            sp = (int)uu((uint32_t)(sp - consumed));
            em &= ~taken;
        }
        if (GS != 64 && refill) {   // the sub-group's cursor, from its leader lane
            cur = (uint32_t)__shfl((int)cur, (int)lead);
            cur_t = __shfl(cur_t, (int)lead);
        }
        lp.tick(0);
        const bool walking = (__ballot(cur != INVALID) & segmask) != 0;
        if (!walking && Tp == 0) {
            done = true;
            continue;
        }
        // fetch: this iteration's nodes and the previous iteration's triangles together,
        // one dependent round trip.  The triangle list is read first, and the load
        // registers stay undefined where a lane has no node / triangle (nothing reads
        // them there): zero-filling them let the compiler reuse a register still owed
        // by a node load, so it waited for the nodes before issuing the triangles.
        // (GS = 64 only: in the run-time-width walk, trace_kernel's drain, the
        // zero-filled form keeps its register allocation without spills)
        const bool has_tri = L < Tp;
        uint4 h, a1, a2, a3, a4, a5;
        float4 r0, r1, r2, r3;
        const float4 *rr;
        if constexpr (GS == 64) {
            const uint32_t trec = has_tri ? tlist[pb * TAIL_TRI + L] : 0u;
            if (cur != INVALID) load_node(g, top, UP ? cur & WIDE_NODE_MASK : cur, h, a1, a2, a3, a4, a5);
            if (UP && cur != INVALID) chainw = gld(reinterpret_cast<const uint32_t *>(g.wnodes + (size_t)g.wstride * (cur & WIDE_NODE_MASK)) + 24 + k);
            rr = g.wtri + 4 * (size_t)trec;
            if (has_tri) { r0 = gld(rr); r1 = gld(rr + 1); r2 = gld(rr + 2); r3 = gld(rr + 3); }
            lp.wait_loads();
            lp.tick(1);
        } else {
            h = make_uint4(0u, 0u, 0u, 0u); a1 = h; a2 = h; a3 = h; a4 = h; a5 = h;
            if (cur != INVALID) load_node(g, top, UP ? cur & WIDE_NODE_MASK : cur, h, a1, a2, a3, a4, a5);
            if (UP && cur != INVALID)
                chainw = gld(reinterpret_cast<const uint32_t *>(g.wnodes + (size_t)g.wstride * (cur & WIDE_NODE_MASK)) + 24 + k);
            r0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f); r1 = r0; r2 = r0; r3 = r0;
            rr = nullptr;
            if (has_tri) {
                rr = g.wtri + 4 * (size_t)tlist[pb * TAIL_TRI + L];
                r0 = gld(rr); r1 = gld(rr + 1); r2 = gld(rr + 2); r3 = gld(rr + 3);
            }
        }
        // expand: sub-group j's 8 lanes slab-test the 8 children of its node
        bool inner = false, leafhit = false;
        float tk = 0.0f;
        uint32_t kind = 0, child = 0, first = 0;
        const bool more = UP && cur != INVALID && (cur & WIDE_CHAIN_MORE) != 0u;
        if (cur != INVALID) {
            const V3 org = v3(__uint_as_float(h.x), __uint_as_float(h.y), __uint_as_float(h.z));
            const float sx = exp_scale(h.w), sy = exp_scale(h.w >> 8), sz = exp_scale(h.w >> 16);
            const int kk = (int)k;
            kind = byte_of(a4.z, a4.w, kk);
            if (UP && (cur & WIDE_ANCESTOR) != 0u && ((cur >> 28) & 7u) == k) kind = 0u;   // the chain's child
            const float tnx = __builtin_fmaf(__builtin_fmaf(byte_f(r.negx ? a2.z : a1.x, r.negx ? a2.w : a1.y, kk), sx, org.x), r.inx, r.onx);
            const float tfx = __builtin_fmaf(__builtin_fmaf(byte_f(r.negx ? a1.x : a2.z, r.negx ? a1.y : a2.w, kk), sx, org.x), r.inx, r.ofx);
            const float tny = __builtin_fmaf(__builtin_fmaf(byte_f(r.negy ? a3.x : a1.z, r.negy ? a3.y : a1.w, kk), sy, org.y), r.iny, r.ony);
            const float tfy = __builtin_fmaf(__builtin_fmaf(byte_f(r.negy ? a1.z : a3.x, r.negy ? a1.w : a3.y, kk), sy, org.y), r.iny, r.ofy);
            const float tnz = __builtin_fmaf(__builtin_fmaf(byte_f(r.negz ? a3.z : a2.x, r.negz ? a3.w : a2.y, kk), sz, org.z), r.inz, r.onz);
            const float tfz = __builtin_fmaf(__builtin_fmaf(byte_f(r.negz ? a2.x : a3.z, r.negz ? a2.y : a3.w, kk), sz, org.z), r.inz, r.ofz);
            const float tmin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(tnx, tny), tnz), 0.0f);
            const float tmax = __builtin_fminf(__builtin_fminf(tfx, tfy), tfz);
            const bool hit = (kind != 0u) & !(tmin > tmax) & !(tmin > cut);
            inner = hit & (kind == WIDE_INNER);
            leafhit = hit & (kind != WIDE_INNER);
            tk = tmin;
            const uint32_t off = byte_of(a5.x, a5.y, kk);
            child = a4.x + off;
            first = a4.y + off;
        }
        // each sub-group continues with its nearest inner child (first of the
        // smallest entry distance) and pushes the others
        const unsigned long long key =
            dpp_min8(inner ? (((unsigned long long)__float_as_uint(tk) << 32) | k) : NONE);
        uint32_t near = INVALID;
        float near_t = 0.0f;
        if (key != NONE) {
            near = a4.x + byte_of(a5.x, a5.y, (int)(key & 7u));
            near_t = __uint_as_float((uint32_t)(key >> 32));
        }
        const bool push = inner && (key & 7u) != k;
        const unsigned long long pm = __ballot(push) & segmask;
        const int pos = sp + __popcll(pm & below);
        if (push && pos < cap) {
            stk[2 * pos] = child;
            stk[2 * pos + 1] = __float_as_uint(tk);
        }
        const int npush = __popcll(pm);
        if (sp + npush > cap) {
            if (L == 0) overflow += (uint32_t)(sp + npush - cap);
            sp = cap;
        } else {
            sp += npush;
        }
        if constexpr (UP) {   // a chain onto the segment's stack (walk_lone<true>)
            const bool cpush = more && chainw != WIDE_NO_PARENT;
            const unsigned long long cm = __ballot(cpush) & segmask;
            if (cm) {
                const int nc = __popcll(cm);
                const int cpos = sp + nc - 1 - __popcll(cm & below);
                if (cpush && cpos < cap) {
                    stk[2 * cpos] = chainw;
                    stk[2 * cpos + 1] = 0u;
                }
                if (sp + nc > cap) {
                    if (L == 0) overflow += (uint32_t)(sp + nc - cap);
                    sp = cap;
                } else {
                    sp += nc;
                }
            }
        }
        cur = near;
        cur_t = near_t;
        // this iteration's hit-leaf triangles, listed in lane order for the next fetch
        const uint32_t cnt = leafhit ? kind : 0u;
        const unsigned long long b0 = __ballot(cnt & 1u) & segmask, b1 = __ballot(cnt & 2u) & segmask,
                                 b2 = __ballot(cnt & 4u) & segmask;
        const uint32_t pre = __popcll(b0 & below) + 2u * __popcll(b1 & below) + 4u * __popcll(b2 & below);
        const uint32_t Tn = __popcll(b0) + 2u * __popcll(b1) + 4u * __popcll(b2);
        // (a leaf holds at most 4 triangles)
        if (cnt > 0u) tlist[(pb ^ 1) * TAIL_TRI + pre] = first;
        if (cnt > 1u) tlist[(pb ^ 1) * TAIL_TRI + pre + 1] = first + 1u;
        if (cnt > 2u) tlist[(pb ^ 1) * TAIL_TRI + pre + 2] = first + 2u;
        if (cnt > 3u) tlist[(pb ^ 1) * TAIL_TRI + pre + 3] = first + 3u;
        lp.tick(2);
        // test the previous iteration's triangles (entries beyond the segment's
        // lanes, rare, are fetched now)
        float lbest = best, lbd = best_bd;
        uint32_t lrank = best_rank;
        int lid = -1;
        for (uint32_t i = L; i < Tp; i += (uint32_t)Gs) {
            if (i != L) {
                rr = g.wtri + 4 * (size_t)tlist[pb * TAIL_TRI + i];
                r0 = gld(rr); r1 = gld(rr + 1); r2 = gld(rr + 2); r3 = gld(rr + 3);
            }
            const uint32_t id = __float_as_uint(r2.y);
            float dist;
            if (id == last ||
                !intersect_record(o, d, r0, r1, r2, dist))
                continue;
            const uint32_t rank = __float_as_uint(r2.z);
            if (!ref_may_beat(dist, rank, lbest, lrank, lbd)) continue;
            V3 lo, hi;
            node_bounds(g, make_uint4(__float_as_uint(r2.w), __float_as_uint(r3.x), __float_as_uint(r3.y), 0u), lo, hi);
            float bd;
            if (!intersect_box(noid, inv, lo, hi, bd) || !ref_beats(dist, rank, bd, lbest, lrank, lbd))
                continue;   // mesh.h:94-96
            lbest = dist;
            lbd = bd;
            lrank = rank;
            lid = rec_of(g, rr);
        }
        __builtin_amdgcn_wave_barrier();   // list reads land before the next iteration's writes
        // the segment's winner (ref_merge): usually no lane or one lane has a hit
        const unsigned long long hm = __ballot(lid != -1) & segmask;
        if (hm != 0) {
            RefHit w = lid == -1 ? RefHit{__builtin_inff(), __builtin_inff(), NONE32, -1} : RefHit{lbest, lbd, lrank, lid};
            if ((hm & (hm - 1)) == 0) {
                const int src = __ffsll((long long)hm) - 1;
                if (GS == 64) {   // src is wave-uniform: scalar reads of the winning lane
                    w = RefHit{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(w.d), src)),
                               __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w.bd), src)),
                               (uint32_t)__builtin_amdgcn_readlane((int)w.rank, src), __builtin_amdgcn_readlane(w.id, src)};
                } else {
                    w = RefHit{__shfl(w.d, src), __shfl(w.bd, src), (uint32_t)__shfl((int)w.rank, src), __shfl(w.id, src)};
                }
            } else {
                for (int off = 1; off < Gs; off <<= 1) w = ref_merge(w, shfl_xor_hit(w, off));
            }
            best = ufl(w.d);
            best_bd = ufl(w.bd);
            best_rank = uu(w.rank);
            best_id = (int)uu((uint32_t)w.id);
            cut = ufl(ref_cut(best, best_bd));
        }
        Tp = uu(Tn);
        sp = (int)uu((uint32_t)sp);
        pb ^= 1;
        lp.tick(3);
        if (cur != INVALID && cur_t > cut) cur = INVALID;
    }
    lp.flush();
    min_distance = best_id == -1 ? -1.0f : best;
    return best_id;
}

// The tail's lone long-lived photon: one walk on the whole wave, 8 cursors of 8
// lanes (lane k of a cursor's sub-group slab-tests child k), software-pipelined.
// walk_segment<64> spends each iteration in sequence: refill the empty cursors
// from the stack, fetch (nodes + the previous iteration's triangles, one round
// trip), expand, test the triangles -- measured (profile build, r04 dp1): 13% /
// 40% / 29% / 18% of 3,244 cycles.  Here the loads of the next iteration are
// issued as soon as they are known -- the nodes of the cursors that descend
// (near child) and the triangles just listed -- and the previous triangles'
// tests, the hit reduction, the culling and the stack refill run while they are
// in flight; only a cursor refilled from the stack issues its node load after
// them.  Same culling rule (a best never below the final one, strict '>'), same
// (distance, reference rank) minimum: the result is walk_segment's.
// Also cheaper per iteration: 32-bit near-child keys (the entry distance's bits
// with the child slot in the low 3 bits: the pick among children whose entries
// differ in those bits only may change, the culling distance is rounded down),
// byte extraction with v_perm.
// Device profile (CHR_PROF_LONE_*): walk_lone ticks REFILL (the stack refill and the
// next nodes' issue), EXPAND (the expansion, including the wait for its nodes) and
// TRIS (the tests, including the wait for their records); FETCH stays 0 -- its loads
// are waited for inside EXPAND and TRIS.  walk_segment ticks all four in sequence.
__device__ __forceinline__ uint32_t byte8(uint32_t lo4, uint32_t hi4, uint32_t k) {   // byte k of (hi4:lo4)
    return __builtin_amdgcn_perm(hi4, lo4, 0x0c0c0c00u | k);
}
// walk_lone loads only the first 8 bytes of a node's last 16 (its slot offsets;
// the rest is pad), and of a triangle record's last 16 the 8 the leaf box needs:
// registers written by an in-flight load but never read are reused by the register
// allocator as temporaries, and the compiler then waits for the load first.
// best / best_rank / best_id: a hit already found seeds the walk (trace_kernel's
// drain of a walk begun lane by lane), as in walk_segment.
// UP (walk_up): the walk starts at node `start` (the leaf node of the photon's
// previous hit: the ray starts on that triangle, and its next hit is usually
// close) and climbs -- start's ancestors (its slot's chain words, wide_bvh.h) go on
// the stack with their entry distance 0, each expanded without the child the
// chain came from, the 8th of a chain continuing it.  Every node of the tree is
// then reached exactly once (start's subtree, plus each ancestor's other
// children), with the same culling: the same tested set as from the root, in
// ~half the dependent iterations for the tail's long-lived photons.
template <bool UP = false, class M>
__device__ __forceinline__ int walk_lone(const DevGeom &g, V3 o, V3 d, uint32_t last, M stk, int cap, M tlist,
                                         uint32_t &overflow, float &min_distance, uint32_t &iters,
                                         float best = __builtin_inff(), uint32_t best_rank = 0xFFFFFFFFu,
                                         int best_id = -1, float best_bd = __builtin_inff(), uint32_t start = 0u,
                                         bool have_pre = false, uint32_t pre_cur = 0xFFFFFFFFu,
                                         uint32_t pre_push = 0xFFFFFFFFu) {
    constexpr uint32_t INVALID = 0xFFFFFFFFu;
    auto ufl = [](float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); };
    auto uu = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };
    o = v3(ufl(o.x), ufl(o.y), ufl(o.z));
    d = v3(ufl(d.x), ufl(d.y), ufl(d.z));
    last = uu(last);
    best = ufl(best);
    best_rank = uu(best_rank);
    best_id = (int)uu((uint32_t)best_id);
    best_bd = ufl(best_bd);
    float cut = ufl(ref_cut(best, best_bd));   // the culling threshold (ref_cut)
    const uint32_t lane = __lane_id();
    const uint32_t k = lane & 7u;                     // child slot of this lane
    const uint32_t lead = lane & ~7u;                 // its sub-group's first lane
    const unsigned long long below = (1ull << lane) - 1ull;
    const V3 noid = v3(-o.x / d.x, -o.y / d.y, -o.z / d.z);
    const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const RaySlab r = make_slab(o, noid, inv);
    uint32_t cur = lane < 8u ? (UP ? start : 0u) : INVALID;   // cursor 0 starts at the root (UP: at start)
    // UP with start's chain already read (have_pre, the tail's prefetch): cursor c > 0
    // starts at the ancestor word pre_cur (start's c-th ancestor, lane-wise; INVALID:
    // none), the 8th (pre_push) goes on the stack, and start pushes no chain of its own
    const bool pre = UP && have_pre;
    if (pre) cur = lane < 8u ? (start & ~WIDE_CHAIN_MORE) : pre_cur;
    uint32_t chainw = INVALID;                        // UP: ancestor word k of the cursor's node (lane k)
    float cur_t = 0.0f;
    int sp = 0;
    if (pre && (pre_push & WIDE_ANCESTOR) != 0u) {   // the 8th ancestor (a valid word), entry distance 0
        if (lane == 0) { stk[0] = pre_push; stk[1] = 0u; }
        __builtin_amdgcn_wave_barrier();
        sp = 1;
    }
    uint32_t Tp = 0;                                  // triangles in flight (listed by the last expansion)
    int pb = 0;                                       // the list buffer they were read from
    iters = 0;
    LoneProf<true> lp;
    uint4 h, a1, a2, a3, a4;                          // the cursor's node (in flight at the loop top)
    uint2 a5;
    float4 r0, r1, r2;                                // this lane's listed triangle (in flight)
    float2 r3;
    const float4 *rr = g.wtri;
    // Every lane issues the same number of loads every iteration (a lane without a
    // cursor loads the root, one without a listed triangle record 0): with a fixed
    // count of younger loads the compiler waits for exactly the older ones
    // (vmcnt(N) instead of vmcnt(0)), so a node fetch overlaps the triangle tests and
    // a triangle fetch the next expansion.  (No LDS copy of the tree top here: a
    // lane-divergent LDS / global choice makes that count unknown.)
    auto fetch_node = [&](uint32_t node) {
        const uint4 *np = g.wnodes + (size_t)g.wstride * (node == INVALID ? 0u : (UP ? node & WIDE_NODE_MASK : node));
        h = gld(np); a1 = gld(np + 1); a2 = gld(np + 2); a3 = gld(np + 3); a4 = gld(np + 4);
        a5 = gld_lo2(np + 5);
        if constexpr (UP) chainw = gld(reinterpret_cast<const uint32_t *>(np) + 24 + k);   // the slot's chain
    };
    auto fetch_tri = [&](uint32_t trec) {
        rr = g.wtri + 4 * (size_t)trec;
        r0 = gld(rr); r1 = gld(rr + 1); r2 = gld(rr + 2);
        const uint2 w = gld_lo2(rr + 3);
        r3 = make_float2(__uint_as_float(w.x), __uint_as_float(w.y));
    };
    fetch_node(cur);
    __builtin_amdgcn_sched_barrier(0);   // nodes before triangles, as in the loop (one wait pattern)
    fetch_tri(0u);   // (none listed yet: the same load pattern as every iteration's end)
    while (true) {
        iters++;
        lp.begin();
        // expand: sub-group j's 8 lanes slab-test the 8 children of its node
        bool inner = false, leafhit = false;
        float tk = 0.0f;
        uint32_t kind = 0, child = 0, first = 0;
        // UP: an ancestor is expanded without the child its chain came from; a chain's
        // last known node pushes its own chain
        const bool more = UP && cur != INVALID && (cur & WIDE_CHAIN_MORE) != 0u;
        if (cur != INVALID) {
            const V3 org = v3(__uint_as_float(h.x), __uint_as_float(h.y), __uint_as_float(h.z));
            const float sx = exp_scale(h.w), sy = exp_scale(h.w >> 8), sz = exp_scale(h.w >> 16);
            kind = byte8(a4.z, a4.w, k);
            if (UP && (cur & WIDE_ANCESTOR) != 0u && ((cur >> 28) & 7u) == k) kind = 0u;
            auto q = [k](uint32_t lo4, uint32_t hi4) { return (float)byte8(lo4, hi4, k); };
            const float tnx = __builtin_fmaf(__builtin_fmaf(q(r.negx ? a2.z : a1.x, r.negx ? a2.w : a1.y), sx, org.x), r.inx, r.onx);
            const float tfx = __builtin_fmaf(__builtin_fmaf(q(r.negx ? a1.x : a2.z, r.negx ? a1.y : a2.w), sx, org.x), r.inx, r.ofx);
            const float tny = __builtin_fmaf(__builtin_fmaf(q(r.negy ? a3.x : a1.z, r.negy ? a3.y : a1.w), sy, org.y), r.iny, r.ony);
            const float tfy = __builtin_fmaf(__builtin_fmaf(q(r.negy ? a1.z : a3.x, r.negy ? a1.w : a3.y), sy, org.y), r.iny, r.ofy);
            const float tnz = __builtin_fmaf(__builtin_fmaf(q(r.negz ? a3.z : a2.x, r.negz ? a3.w : a2.y), sz, org.z), r.inz, r.onz);
            const float tfz = __builtin_fmaf(__builtin_fmaf(q(r.negz ? a2.x : a3.z, r.negz ? a2.y : a3.w), sz, org.z), r.inz, r.ofz);
            const float tmin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(tnx, tny), tnz), 0.0f);
            const float tmax = __builtin_fminf(__builtin_fminf(tfx, tfy), tfz);
            const bool hit = (kind != 0u) & !(tmin > tmax) & !(tmin > cut);
            inner = hit & (kind == WIDE_INNER);
            leafhit = hit & (kind != WIDE_INNER);
            tk = tmin;
            const uint32_t off = byte8(a5.x, a5.y, k);
            child = a4.x + off;
            first = a4.y + off;
        }
        // each sub-group continues with its nearest inner child and pushes the others;
        // key: the entry distance's bits (>= 0: ordered as unsigned) with the slot in the
        // low 3 bits, min over the sub-group by DPP
        uint32_t key = inner ? ((__float_as_uint(tk) & ~7u) | k) : INVALID;
        auto dmin = [](uint32_t v, auto ctrl) {
            const uint32_t o2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, decltype(ctrl)::value, 0xF, 0xF, true);
            return o2 < v ? o2 : v;
        };
        key = dmin(key, std::integral_constant<int, 0xB1>());    // quad_perm [1,0,3,2]
        key = dmin(key, std::integral_constant<int, 0x4E>());    // quad_perm [2,3,0,1]
        key = dmin(key, std::integral_constant<int, 0x141>());   // row_half_mirror
        uint32_t near = INVALID;
        if (key != INVALID) near = a4.x + byte8(a5.x, a5.y, key & 7u);
        const bool push = inner && (key & 7u) != k;
        const unsigned long long pm = __ballot(push);
        const int pos = sp + __popcll(pm & below);
        if (push && pos < cap) {
            stk[2 * pos] = child;
            stk[2 * pos + 1] = __float_as_uint(tk);
        }
        const int npush = __popcll(pm);
        if (sp + npush > cap) {
            if (lane == 0) overflow += (uint32_t)(sp + npush - cap);
            sp = cap;
        } else {
            sp += npush;
        }
        if constexpr (UP) {   // a chain onto the stack, entry distance 0, its first ancestor on top
            const bool cpush = more && chainw != WIDE_NO_PARENT;
            const unsigned long long cm = __ballot(cpush);
            if (cm) {
                const int nc = __popcll(cm);
                const int cpos = sp + nc - 1 - __popcll(cm & below);
                if (cpush && cpos < cap) {
                    stk[2 * cpos] = chainw;
                    stk[2 * cpos + 1] = 0u;
                }
                if (sp + nc > cap) {
                    if (lane == 0) overflow += (uint32_t)(sp + nc - cap);
                    sp = cap;
                } else {
                    sp += nc;
                }
            }
        }
        cur = near;
        cur_t = __uint_as_float(key & ~7u);           // <= the child's entry distance
        // this expansion's hit-leaf triangles, listed in lane order: each lane writes
        // exactly its own entries [pre, pre + cnt) (slot indices clamped to the buffer)
        const uint32_t cnt = leafhit ? kind : 0u;
        const unsigned long long b0 = __ballot(cnt & 1u), b1 = __ballot(cnt & 2u), b2 = __ballot(cnt & 4u);
        const uint32_t pre = __popcll(b0 & below) + 2u * __popcll(b1 & below) + 4u * __popcll(b2 & below);
        const uint32_t Tn = uu(__popcll(b0) + 2u * __popcll(b1) + 4u * __popcll(b2));
        const int nb = (pb ^ 1) * TAIL_TRI;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if ((uint32_t)i < cnt) tlist[nb + (int)min(pre + (uint32_t)i, (uint32_t)(TAIL_TRI - 1))] = first + (uint32_t)i;
        lp.tick(2);
        // cursors without a node take the topmost unculled stack entries (walk_segment's
        // window refill; culled with the best before this iteration's triangle tests --
        // conservative), passed through the previous list's buffer (entries 0..15: its
        // triangles are loaded, only entries >= 64 are still read, below)
        unsigned long long em = __ballot(k == 0u && cur == INVALID);
        while (em != 0 && sp > 0) {
            const int W = sp < 8 ? sp : 8;
            uint32_t en = 0, et = 0;
            bool ok = false;
            if (lane < (uint32_t)W) {
                en = stk[2 * (sp - 1 - (int)lane)];
                et = stk[2 * (sp - 1 - (int)lane) + 1];
                ok = !(__uint_as_float(et) > cut);            // mesh.h:94-96
            }
            const unsigned long long okm = __ballot(ok);
            const int need = __popcll(em), nv = __popcll(okm);
            const int take = need < nv ? need : nv;
            const int rho = __popcll(okm & below);
            const unsigned long long stopm = __ballot(ok && rho == take);
            const int consumed = stopm ? (__ffsll((long long)stopm) - 1) : W;
            if (ok && rho < take) {
                tlist[pb * TAIL_TRI + 2 * rho] = en;
                tlist[pb * TAIL_TRI + 2 * rho + 1] = et;
            }
            __builtin_amdgcn_wave_barrier();
            const bool empty = ((em >> lead) & 1ull) != 0;
            const int rnk = __popcll(em & ((1ull << lead) - 1ull));
            const unsigned long long taken = __ballot(k == 0u && empty && rnk < take);
            if (empty && rnk < take) {
                cur = tlist[pb * TAIL_TRI + 2 * rnk];
                cur_t = __uint_as_float(tlist[pb * TAIL_TRI + 2 * rnk + 1]);
            }
            __builtin_amdgcn_wave_barrier();
            sp = (int)uu((uint32_t)(sp - consumed));
            em &= ~taken;
        }
        sp = (int)uu((uint32_t)sp);
        // every cursor's next node, in flight during the triangle tests below
        fetch_node(cur);
        lp.tick(0);
        // test the previous list's triangles: each lane its own (loaded last
        // iteration); entries beyond the 64 lanes (rare) are fetched in a loop of their
        // own, so the common test waits for nothing in flight
        float lbest = best, lbd = best_bd;
        uint32_t lrank = best_rank;
        int lid = -1;
        // (t3 = nullptr: the leaf-box words are loaded for a candidate only)
        auto test = [&](const float4 &t0, const float4 &t1, const float4 &t2, const float2 *t3, const float4 *tr) {
            const uint32_t id = __float_as_uint(t2.y);
            float dist;
            if (id == last || !intersect_record(o, d, t0, t1, t2, dist)) return;
            const uint32_t rank = __float_as_uint(t2.z);
            if (!ref_may_beat(dist, rank, lbest, lrank, lbd)) return;
            uint2 w;
            if (t3) w = make_uint2(__float_as_uint(t3->x), __float_as_uint(t3->y));
            else w = gld_lo2(tr + 3);
            V3 lo, hi;
            node_bounds(g, make_uint4(__float_as_uint(t2.w), w.x, w.y, 0u), lo, hi);
            float bd;
            if (!intersect_box(noid, inv, lo, hi, bd) || !ref_beats(dist, rank, bd, lbest, lrank, lbd))
                return;   // mesh.h:94-96
            lbest = dist;
            lbd = bd;
            lrank = rank;
            lid = rec_of(g, tr);
        };
        if (lane < Tp) {
            // every word of the lane's triangle waited for here, with the node loads
            // above still in flight: a register the allocator reuses later is then
            // no longer owed by a load (the compiler would wait for everything there)
            asm volatile("" :: "v"(r3.x), "v"(r3.y));
            test(r0, r1, r2, &r3, rr);
        }
        for (uint32_t i = lane + 64u; i < Tp; i += 64u) {
            const float4 *tr = g.wtri + 4 * (size_t)tlist[pb * TAIL_TRI + (int)i];
            test(gld(tr), gld(tr + 1), gld(tr + 2), nullptr, tr);
        }
        // the wave's winner (ref_merge): usually no lane or one lane has a hit
        const unsigned long long hm = __ballot(lid != -1);
        if (hm != 0) {
            RefHit w = lid == -1 ? RefHit{__builtin_inff(), __builtin_inff(), NONE32, -1} : RefHit{lbest, lbd, lrank, lid};
            if ((hm & (hm - 1)) == 0) {
                const int src = __ffsll((long long)hm) - 1;
                w = RefHit{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(w.d), src)),
                           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w.bd), src)),
                           (uint32_t)__builtin_amdgcn_readlane((int)w.rank, src), __builtin_amdgcn_readlane(w.id, src)};
            } else {
                for (int off = 1; off < 64; off <<= 1) w = ref_merge(w, shfl_xor_hit(w, off));
            }
            best = ufl(w.d);
            best_bd = ufl(w.bd);
            best_rank = uu(w.rank);
            best_id = (int)uu((uint32_t)w.id);
            cut = ufl(ref_cut(best, best_bd));
        }
        // this expansion's triangles, in flight during the stack refill and the next
        // expansion (the registers of the ones just tested are free)
        __builtin_amdgcn_wave_barrier();
        fetch_tri(lane < Tn ? tlist[nb + (int)lane] : 0u);
        Tp = Tn;
        pb ^= 1;
        if (cur != INVALID && cur_t > cut) cur = INVALID;   // its node load is in flight: ignored
        lp.tick(3);
        if (__ballot(cur != INVALID) == 0 && Tp == 0 && sp == 0) break;
    }
    lp.flush();
    min_distance = best_id == -1 ? -1.0f : best;
    return best_id;
}

// ---------------------------------------------------------------- pair walk
// The lone walk on two waves of a workgroup (two SIMDs): the WALKER runs the
// node expansions, the stack and the refills, and lists each iteration's
// hit-leaf triangles into a ring of two LDS buffers; the TESTER, another wave of
// the workgroup with no photon of its own, tests the listed triangles and
// publishes the running (distance, reference rank) minimum, which the walker
// culls with.  walk_lone does both in one instruction stream (~2,300 shader
// cycles per iteration, bound by its own issue, §11.7); split, each wave issues
// about half of it per iteration.  The tester's best lags the walker by about
// an iteration -- never below the final one, so culling stays conservative -- and
// the result is the min over every listed triangle with the reference leaf-box
// check, as in walk_lone / walk_segment.
// The mailbox (PB_* words, LDS, one per workgroup) carries the ray and the
// handshake: the walker posts (PS_REQ), a helper takes it (PS_TAKEN), lists
// count up in PB_WSEQ, the tester's progress in PB_TREAD (lists read: the
// walker may reuse that buffer) and PB_TSEQ (lists tested), the walker's end in
// PB_WDONE, the tester's in PS_DONE.  Every wait is bounded (PAIR_SPIN_MAX
// polls): a lost handshake -- a timed-out wait, an abort, or a tester that did
// not test every list (PB_TSEQ != lists published) -- is reported to the caller,
// which walks the ray again alone (walk_lone), and is counted (1 << 20 in the
// stack-overflow counter); PB_ABORT then stays set and the workgroup pairs no
// more walks (an abandoned tester may still be reading the box).
enum : int {
    PB_STATE, PB_IDLE, PB_WORKERS, PB_WSEQ, PB_WDONE, PB_TREAD, PB_TSEQ, PB_BEST, PB_RANK, PB_ID,
    PB_OX, PB_OY, PB_OZ, PB_DX, PB_DY, PB_DZ, PB_LAST, PB_CNT0, PB_CNT1, PB_LISTS, PB_ABORT,
    PB_BD, PB_CUT,   // the best's leaf-box entry and the culling threshold (ref_cut) the walker reads
    PB_WORDS = 24
};
enum : uint32_t { PS_IDLE = 0, PS_POSTING = 1, PS_REQ = 2, PS_TAKEN = 3, PS_DONE = 4, PS_EXIT = 5 };
constexpr uint32_t PAIR_SPIN_MAX = 1u << 21;
__device__ __forceinline__ uint32_t lds_ld(CHR_LDS uint32_t *p) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)*(volatile CHR_LDS uint32_t *)p);
}
__device__ __forceinline__ void lds_st(CHR_LDS uint32_t *p, uint32_t v) {   // lane 0 writes
    if (__lane_id() == 0) *(volatile CHR_LDS uint32_t *)p = v;
}
__device__ __forceinline__ void lds_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); }
__device__ __forceinline__ void lds_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); }
// poll until pred() (wave-uniform), at most PAIR_SPIN_MAX times; false on timeout
template <class P>
__device__ __forceinline__ bool pair_wait(CHR_LDS uint32_t *box, uint32_t spin, P pred) {
    for (uint32_t i = 0; i < spin; ++i) {
        if (pred()) return true;
        if (lds_ld(box + PB_ABORT)) return false;
        __builtin_amdgcn_s_sleep(1);
    }
    lds_st(box + PB_ABORT, 1u);
    return false;
}

// The walker (whole wave, converged).  lists: this wave's 2 x TAIL_TRI words;
// stk: cap entries of stack, the last 8 of them used as the refill's scratch.
// The box must have been posted (ray, seed best, PB_LISTS) by this wave.
template <class M>
__device__ __forceinline__ int walk_pair_walker(const DevGeom &g, const TopNodes &top, V3 o, V3 d, M stk, int cap,
                                                CHR_LDS uint32_t *lists, CHR_LDS uint32_t *box, uint32_t spin,
                                                uint32_t &overflow, float &min_distance, uint32_t &iters, bool &lost) {
    constexpr uint32_t INVALID = 0xFFFFFFFFu;
    auto ufl = [](float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); };
    auto uu = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };
    o = v3(ufl(o.x), ufl(o.y), ufl(o.z));
    d = v3(ufl(d.x), ufl(d.y), ufl(d.z));
    const int scap = cap - 8;                         // stack entries; [scap, cap): the refill's scratch
    const uint32_t lane = __lane_id();
    const uint32_t k = lane & 7u;
    const uint32_t lead = lane & ~7u;
    const unsigned long long below = (1ull << lane) - 1ull;
    const V3 noid = v3(-o.x / d.x, -o.y / d.y, -o.z / d.z);
    const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const RaySlab r = make_slab(o, noid, inv);
    uint32_t cur = lane < 8u ? 0u : INVALID;
    float cur_t = 0.0f;
    int sp = 0;
    uint32_t nl = 0;                                  // lists published
    bool ok = true;
    iters = 0;
    // a node's 88 used bytes (the last 16-byte word's first 8: its slot offsets), from
    // the LDS top of the tree or global memory: every register a load writes is read
    // by the expansion, so none is reused as a temporary while the load is in flight
    // (the compiler would wait for every load there)
    uint4 h, a1, a2, a3, a4;
    uint2 a5;
    auto fetch_node = [&](uint32_t node) {
        if (node < top.n) {
            const CHR_LDS u32x4 *tp = top.p + 6u * node;
            h = u4(tp[0]); a1 = u4(tp[1]); a2 = u4(tp[2]); a3 = u4(tp[3]); a4 = u4(tp[4]);
            const chr_u32x2 t5 = *(const CHR_LDS chr_u32x2 *)(tp + 5);
            a5 = make_uint2(t5.x, t5.y);
        } else {
            const uint4 *np = g.wnodes + (size_t)g.wstride * node;
            h = gld(np); a1 = gld(np + 1); a2 = gld(np + 2); a3 = gld(np + 3); a4 = gld(np + 4);
            a5 = gld_lo2(np + 5);
        }
    };
    fetch_node(cur == INVALID ? 0u : cur);
    float cut = __uint_as_float(lds_ld(box + PB_CUT));   // the tester's culling threshold, read once per iteration
    while (true) {
        iters++;
        bool inner = false, leafhit = false;
        float tk = 0.0f;
        uint32_t kind = 0, child = 0, first = 0;
        if (cur != INVALID) {
            const V3 org = v3(__uint_as_float(h.x), __uint_as_float(h.y), __uint_as_float(h.z));
            const float sx = exp_scale(h.w), sy = exp_scale(h.w >> 8), sz = exp_scale(h.w >> 16);
            kind = byte8(a4.z, a4.w, k);
            auto q = [k](uint32_t lo4, uint32_t hi4) { return (float)byte8(lo4, hi4, k); };
            const float tnx = __builtin_fmaf(__builtin_fmaf(q(r.negx ? a2.z : a1.x, r.negx ? a2.w : a1.y), sx, org.x), r.inx, r.onx);
            const float tfx = __builtin_fmaf(__builtin_fmaf(q(r.negx ? a1.x : a2.z, r.negx ? a1.y : a2.w), sx, org.x), r.inx, r.ofx);
            const float tny = __builtin_fmaf(__builtin_fmaf(q(r.negy ? a3.x : a1.z, r.negy ? a3.y : a1.w), sy, org.y), r.iny, r.ony);
            const float tfy = __builtin_fmaf(__builtin_fmaf(q(r.negy ? a1.z : a3.x, r.negy ? a1.w : a3.y), sy, org.y), r.iny, r.ofy);
            const float tnz = __builtin_fmaf(__builtin_fmaf(q(r.negz ? a3.z : a2.x, r.negz ? a3.w : a2.y), sz, org.z), r.inz, r.onz);
            const float tfz = __builtin_fmaf(__builtin_fmaf(q(r.negz ? a2.x : a3.z, r.negz ? a2.y : a3.w), sz, org.z), r.inz, r.ofz);
            const float tmin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(tnx, tny), tnz), 0.0f);
            const float tmax = __builtin_fminf(__builtin_fminf(tfx, tfy), tfz);
            const bool hit = (kind != 0u) & !(tmin > tmax) & !(tmin > cut);
            inner = hit & (kind == WIDE_INNER);
            leafhit = hit & (kind != WIDE_INNER);
            tk = tmin;
            const uint32_t off = byte8(a5.x, a5.y, k);
            child = a4.x + off;
            first = a4.y + off;
        }
        // near child (walk_lone's 32-bit keys) and pushes
        uint32_t key = inner ? ((__float_as_uint(tk) & ~7u) | k) : INVALID;
        auto dmin = [](uint32_t v, auto ctrl) {
            const uint32_t o2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, decltype(ctrl)::value, 0xF, 0xF, true);
            return o2 < v ? o2 : v;
        };
        key = dmin(key, std::integral_constant<int, 0xB1>());
        key = dmin(key, std::integral_constant<int, 0x4E>());
        key = dmin(key, std::integral_constant<int, 0x141>());
        uint32_t near = INVALID;
        if (key != INVALID) near = a4.x + byte8(a5.x, a5.y, key & 7u);
        const bool push = inner && (key & 7u) != k;
        const unsigned long long pm = __ballot(push);
        const int pos = sp + __popcll(pm & below);
        if (push && pos < scap) {
            stk[2 * pos] = child;
            stk[2 * pos + 1] = __float_as_uint(tk);
        }
        const int npush = __popcll(pm);
        if (sp + npush > scap) {
            if (lane == 0) overflow += (uint32_t)(sp + npush - scap);
            sp = scap;
        } else {
            sp += npush;
        }
        cur = near;
        cur_t = __uint_as_float(key & ~7u);
        // this expansion's hit-leaf triangles -> list nl (buffer nl & 1, free once the
        // tester has read list nl - 2), published once the next nodes are in flight
        const uint32_t cnt = leafhit ? kind : 0u;
        const unsigned long long b0 = __ballot(cnt & 1u), b1 = __ballot(cnt & 2u), b2 = __ballot(cnt & 4u);
        const uint32_t Tn = uu(__popcll(b0) + 2u * __popcll(b1) + 4u * __popcll(b2));
        // cursors without a node take the topmost unculled stack entries (walk_lone's refill)
        unsigned long long em = __ballot(k == 0u && cur == INVALID);
        while (em != 0 && sp > 0) {
            const int W = sp < 8 ? sp : 8;
            uint32_t en = 0, et = 0;
            bool okk = false;
            if (lane < (uint32_t)W) {
                en = stk[2 * (sp - 1 - (int)lane)];
                et = stk[2 * (sp - 1 - (int)lane) + 1];
                okk = !(__uint_as_float(et) > cut);            // mesh.h:94-96
            }
            const unsigned long long okm = __ballot(okk);
            const int need = __popcll(em), nv = __popcll(okm);
            const int take = need < nv ? need : nv;
            const int rho = __popcll(okm & below);
            const unsigned long long stopm = __ballot(okk && rho == take);
            const int consumed = stopm ? (__ffsll((long long)stopm) - 1) : W;
            if (okk && rho < take) {
                stk[2 * (scap + rho)] = en;
                stk[2 * (scap + rho) + 1] = et;
            }
            __builtin_amdgcn_wave_barrier();
            const bool empty = ((em >> lead) & 1ull) != 0;
            const int rnk = __popcll(em & ((1ull << lead) - 1ull));
            const unsigned long long taken = __ballot(k == 0u && empty && rnk < take);
            if (empty && rnk < take) {
                cur = stk[2 * (scap + rnk)];
                cur_t = __uint_as_float(stk[2 * (scap + rnk) + 1]);
            }
            __builtin_amdgcn_wave_barrier();
            sp = (int)uu((uint32_t)(sp - consumed));
            em &= ~taken;
        }
        sp = (int)uu((uint32_t)sp);
        if (cur != INVALID && cur_t > cut) cur = INVALID;
        const bool end = __ballot(cur != INVALID) == 0 && sp == 0;
        if (!end) fetch_node(cur == INVALID ? 0u : cur);
        if (Tn) {
            const uint32_t pre = __popcll(b0 & below) + 2u * __popcll(b1 & below) + 4u * __popcll(b2 & below);
            if (nl >= 2u && ok) ok = pair_wait(box, spin, [&]() { return lds_ld(box + PB_TREAD) + 1u >= nl; });
            const int nb = (int)(nl & 1u) * TAIL_TRI;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if ((uint32_t)i < cnt) lists[nb + (int)min(pre + (uint32_t)i, (uint32_t)(TAIL_TRI - 1))] = first + (uint32_t)i;
            lds_st(box + PB_CNT0 + (nl & 1u), Tn);
            lds_release();
            lds_st(box + PB_WSEQ, nl + 1u);
            nl++;
        }
        cut = __uint_as_float(lds_ld(box + PB_CUT));
        if (end) break;
    }
    lds_release();
    lds_st(box + PB_WDONE, nl);
    if (ok) ok = pair_wait(box, spin, [&]() { return lds_ld(box + PB_STATE) == PS_DONE; });
    lds_acquire();
    // the tester's minimum covers every list only if it tested all nl of them and no
    // side gave up (a tester whose wait timed out also ends with PS_DONE)
    if (ok) ok = lds_ld(box + PB_TSEQ) == nl && lds_ld(box + PB_ABORT) == 0u;
    const float fbest = __uint_as_float(lds_ld(box + PB_BEST));
    const int best_id = (int)lds_ld(box + PB_ID);
    if (!ok && lane == 0) overflow += 1u << 20;   // a lost handshake: counted with the stack overflows
    lost = !ok;
    min_distance = best_id == -1 ? -1.0f : fbest;
    return best_id;
}

// The tester (whole wave, converged), after taking a posted box: tests every
// list the walker publishes until the walker's end, then PS_DONE.  lbase: the
// LDS word base PB_LISTS is relative to.
__device__ __forceinline__ void walk_pair_tester(const DevGeom &g, CHR_LDS uint32_t *box, CHR_LDS uint32_t *lbase,
                                                 uint32_t spin) {
    const uint32_t lane = __lane_id();
    const V3 o = v3(__uint_as_float(lds_ld(box + PB_OX)), __uint_as_float(lds_ld(box + PB_OY)),
                    __uint_as_float(lds_ld(box + PB_OZ)));
    const V3 d = v3(__uint_as_float(lds_ld(box + PB_DX)), __uint_as_float(lds_ld(box + PB_DY)),
                    __uint_as_float(lds_ld(box + PB_DZ)));
    const uint32_t last = lds_ld(box + PB_LAST);
    CHR_LDS uint32_t *lists = lbase + lds_ld(box + PB_LISTS);
    float best = __uint_as_float(lds_ld(box + PB_BEST)), best_bd = __uint_as_float(lds_ld(box + PB_BD));
    uint32_t best_rank = lds_ld(box + PB_RANK);
    int best_id = (int)lds_ld(box + PB_ID);
    const V3 noid = v3(-o.x / d.x, -o.y / d.y, -o.z / d.z);
    const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    for (uint32_t j = 0;; ++j) {
        uint32_t ws = 0;
        const bool ok = pair_wait(box, spin, [&]() {
            const uint32_t wd = lds_ld(box + PB_WDONE);
            ws = lds_ld(box + PB_WSEQ);
            return ws > j || wd == j;
        });
        if (!ok || ws <= j) break;   // the walker's end: every list tested
        lds_acquire();
        // bounded reads whatever the buffers hold: after a lost handshake the walker
        // reuses them as walk_lone's scratch while this wave may still be reading
        const uint32_t n = min(lds_ld(box + PB_CNT0 + (j & 1u)), (uint32_t)TAIL_TRI);
        const int nb = (int)(j & 1u) * TAIL_TRI;
        auto rec = [&](uint32_t i) { const uint32_t t = lists[nb + (int)i]; return t < g.nwtri ? t : 0u; };
        const uint32_t trec = lane < n ? rec(lane) : 0u;
        // the list is in registers: its buffer is free (before the loads, which a
        // release would wait for)
        if (n <= 64u) { lds_release(); lds_st(box + PB_TREAD, j + 1u); }
        const float4 *rr = g.wtri + 4 * (size_t)trec;
        const float4 r0 = gld(rr), r1 = gld(rr + 1), r2 = gld(rr + 2);
        const uint2 w3 = gld_lo2(rr + 3);
        float lbest = best, lbd = best_bd;
        uint32_t lrank = best_rank;
        int lid = -1;
        auto test = [&](const float4 &t0, const float4 &t1, const float4 &t2, uint2 w, const float4 *tr) {
            const uint32_t id = __float_as_uint(t2.y);
            float dist;
            if (id == last || !intersect_record(o, d, t0, t1, t2, dist)) return;
            const uint32_t rank = __float_as_uint(t2.z);
            if (!ref_may_beat(dist, rank, lbest, lrank, lbd)) return;
            V3 lo, hi;
            node_bounds(g, make_uint4(__float_as_uint(t2.w), w.x, w.y, 0u), lo, hi);
            float bd;
            if (!intersect_box(noid, inv, lo, hi, bd) || !ref_beats(dist, rank, bd, lbest, lrank, lbd))
                return;   // mesh.h:94-96
            lbest = dist;
            lbd = bd;
            lrank = rank;
            lid = rec_of(g, tr);
        };
        if (lane < n) test(r0, r1, r2, w3, rr);
        for (uint32_t i = lane + 64u; i < n; i += 64u) {
            const float4 *tr = g.wtri + 4 * (size_t)rec(i);
            test(gld(tr), gld(tr + 1), gld(tr + 2), gld_lo2(tr + 3), tr);
        }
        if (n > 64u) { lds_release(); lds_st(box + PB_TREAD, j + 1u); }
        const unsigned long long hm = __ballot(lid != -1);
        if (hm != 0) {   // the wave's winner (ref_merge)
            RefHit wv = lid == -1 ? RefHit{__builtin_inff(), __builtin_inff(), NONE32, -1} : RefHit{lbest, lbd, lrank, lid};
            for (int off = 1; off < 64; off <<= 1) wv = ref_merge(wv, shfl_xor_hit(wv, off));
            best = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wv.d)));
            best_bd = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wv.bd)));
            best_rank = (uint32_t)__builtin_amdgcn_readfirstlane((int)wv.rank);
            best_id = __builtin_amdgcn_readfirstlane(wv.id);
            lds_st(box + PB_RANK, best_rank);
            lds_st(box + PB_ID, (uint32_t)best_id);
            lds_st(box + PB_BD, __float_as_uint(best_bd));
            lds_st(box + PB_BEST, __float_as_uint(best));
            lds_st(box + PB_CUT, __float_as_uint(ref_cut(best, best_bd)));
        }
        lds_release();
        lds_st(box + PB_TSEQ, j + 1u);
    }
    lds_release();
    // TAKEN -> DONE only: after a lost handshake the walker has moved on and the box
    // may already say something else (PS_EXIT in the timing kernel)
    if (lane == 0) atomicCAS((uint32_t *)box + PB_STATE, PS_TAKEN, PS_DONE);
}

// The walker's side of a pair walk: post the ray into the box (the caller has
// claimed it: PS_POSTING), walk, release the box.  lost: the handshake was lost
// and the result is not the walk's (the caller walks the ray alone); the box
// then stays aborted (never PS_IDLE again), so no walker of the workgroup claims
// it while the abandoned tester may still use it.
template <class M>
__device__ __forceinline__ int walk_pair(const DevGeom &g, const TopNodes &top, V3 o, V3 d, uint32_t last, M stk,
                                         int cap, CHR_LDS uint32_t *lists, uint32_t lists_off, CHR_LDS uint32_t *box,
                                         uint32_t spin, uint32_t &overflow, float &min_distance, uint32_t &iters,
                                         bool &lost) {
    lds_st(box + PB_WSEQ, 0u);
    lds_st(box + PB_WDONE, 0xFFFFFFFFu);
    lds_st(box + PB_TREAD, 0u);
    lds_st(box + PB_TSEQ, 0u);
    lds_st(box + PB_BEST, __float_as_uint(__builtin_inff()));
    lds_st(box + PB_BD, __float_as_uint(__builtin_inff()));
    lds_st(box + PB_CUT, __float_as_uint(__builtin_inff()));
    lds_st(box + PB_RANK, 0xFFFFFFFFu);
    lds_st(box + PB_ID, 0xFFFFFFFFu);
    lds_st(box + PB_OX, __float_as_uint(o.x));
    lds_st(box + PB_OY, __float_as_uint(o.y));
    lds_st(box + PB_OZ, __float_as_uint(o.z));
    lds_st(box + PB_DX, __float_as_uint(d.x));
    lds_st(box + PB_DY, __float_as_uint(d.y));
    lds_st(box + PB_DZ, __float_as_uint(d.z));
    lds_st(box + PB_LAST, last);
    lds_st(box + PB_LISTS, lists_off);
    lds_release();
    lds_st(box + PB_STATE, PS_REQ);
    const int tri = walk_pair_walker(g, top, o, d, stk, cap, lists, box, spin, overflow, min_distance, iters, lost);
    lds_release();
    if (lost) lds_st(box + PB_ABORT, 1u);
    else lds_st(box + PB_STATE, PS_IDLE);
    return tri;
}

// Where a long-lived photon's tail step goes (profile build: CHR_PROF_LONG_*):
// wave cycles per phase of the steps beyond the 64th of each photon, counted by its
// group's first lane.  mark(i) closes phase i at the current clock.
enum { LP_WALK, LP_FILL, LP_TO_BOUNDARY, LP_AT_BOUNDARY, LP_OTHER, LP_N };
template <bool ON>
struct LongProf {
    __device__ __forceinline__ void step(bool) {}
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void flush() {}
};
#ifdef CHR_DEVICE_PROFILE
template <>
struct LongProf<true> {
    unsigned long long cyc[LP_N] = {0ull, 0ull, 0ull, 0ull, 0ull}, steps = 0ull, t = 0ull;
    bool on = false;
    // a step begins (on: this lane's photon is long and walks this step); the time
    // since the last phase closed is OTHER (the loop, the ballots, the walk's set-up)
    __device__ __forceinline__ void step(bool long_walk) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        if (on) cyc[LP_OTHER] += now - t;
        on = long_walk;
        if (on) steps++;
        t = now;
    }
    __device__ __forceinline__ void mark(int i) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        if (on) cyc[i] += now - t;
        t = now;
    }
    __device__ __forceinline__ void flush() {
        prof_add(CHR_PROF_LONG_WALK, steps, cyc[LP_WALK]);
        prof_add(CHR_PROF_LONG_FILL, 0ull, cyc[LP_FILL]);
        prof_add(CHR_PROF_LONG_TO_BOUNDARY, 0ull, cyc[LP_TO_BOUNDARY]);
        prof_add(CHR_PROF_LONG_AT_BOUNDARY, 0ull, cyc[LP_AT_BOUNDARY]);
        prof_add(CHR_PROF_LONG_OTHER, 0ull, cyc[LP_OTHER]);
    }
};
#endif

template <int MINW, bool WIRES = true>
__global__ __launch_bounds__(BLOCK, MINW) void propagate_tail_kernel(const DevGeom *__restrict__ gdev, PropagateArgs a,
                                                                     uint32_t cap) {
    __shared__ uint32_t stacks[(BLOCK / 8) * TAIL_STACK * 2];
    __shared__ uint32_t tris[(BLOCK / 64) * 2 * TAIL_TRI];
    const uint32_t tid = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t lane = __lane_id();
    if (a.mode && *a.mode != a.want) return;
    // a tail overlapped by the next batch (chr_propagate_batches) is the critical
    // path: its waves win the SIMD's issue arbitration over that batch's walk
    if (a.prio) __builtin_amdgcn_s_setprio(3);
    // the workgroup's pair-walk mailbox (walk_pair), ordered before any use by the
    // barriers of phys_cache / stage_top below
    __shared__ uint32_t box_s[PB_WORDS];
    CHR_LDS uint32_t *box = (CHR_LDS uint32_t *)box_s;
    if (threadIdx.x == 0) {
        box_s[PB_STATE] = PS_IDLE;
        box_s[PB_IDLE] = 0u;
        box_s[PB_WORKERS] = BLOCK / 64;
        box_s[PB_ABORT] = 0u;
    }
    CHR_PHYS_LDS(phys_lds, TAIL_PHYS_WORDS);   // phys_lds_bytes(TAIL_PHYS_WORDS) of dynamic LDS
    const DevGeom g = phys_cache(*gdev, phys_lds, TAIL_PHYS_WORDS);
    __shared__ uint4 top_lds[6 * TOP_NODES];   // 7 KB: 2 workgroups per CU hold 2 x 79 KB
    const TopNodes top = stage_top<BLOCK>(g, (CHR_LDS u32x4 *)top_lds, TOP_NODES);
    const uint32_t slot = tid / 8, sub = tid & 7u;
    const uint32_t n = a.dev_n ? *a.dev_n - 1u : (uint32_t)a.nthreads;
    const uint32_t nslot = cap < n ? cap : n;
    // work-queue mode: groups take the next queue position when their photon ends, so the
    // launch is one resident grid (no waves waiting for dispatch behind the first ones,
    // no wave held by its slowest photon while its other groups idle)
    const bool wq = a.work != nullptr && n <= cap;
    // A wave without photons (left) serves as its workgroup's pair-walk tester
    // (walk_pair_tester) until no wave of the workgroup has photons: every wave
    // calls this once, when it leaves the photon loop (or has no slot at all).
    auto serve = [&]() {
        if (lane == 0) atomicSub(&box_s[PB_WORKERS], 1u);
        if (!a.pair) return;
        if (lane == 0) atomicAdd(&box_s[PB_IDLE], 1u);
        while (true) {
            if (lds_ld(box + PB_STATE) == PS_REQ) {
                uint32_t old = 0;
                if (lane == 0) old = atomicCAS(&box_s[PB_STATE], PS_REQ, PS_TAKEN);
                if ((uint32_t)__builtin_amdgcn_readfirstlane((int)old) == PS_REQ) {
                    if (lane == 0) atomicSub(&box_s[PB_IDLE], 1u);
                    lds_acquire();
                    walk_pair_tester(g, box, (CHR_LDS uint32_t *)tris, PAIR_SPIN_MAX);
                    if (lane == 0) atomicAdd(&box_s[PB_IDLE], 1u);
                    continue;
                }
            }
            if (lds_ld(box + PB_WORKERS) == 0u) break;   // no walker left to serve
            __builtin_amdgcn_s_sleep(2);
        }
    };
    if (!wq && (tid & ~63u) / 8 >= nslot) {            // whole waves: the others help walk
        serve();
        return;
    }
    auto next_q = [&]() -> uint32_t {   // the group's next queue position (group-uniform)
        uint32_t v = 0;
        if (sub == 0) v = atomicAdd(a.work, 1u);
        return (uint32_t)__shfl((int)v, (int)(lane & ~7u));
    };
    CHR_LDS uint32_t *wstack = (CHR_LDS uint32_t *)stacks + (threadIdx.x >> 6) * 8 * TAIL_STACK * 2;
    CHR_LDS uint32_t *wtris = (CHR_LDS uint32_t *)tris + (threadIdx.x >> 6) * 2 * TAIL_TRI;
    chr_xorwow rng;
    bool have_rng = false;
    uint32_t overflow = 0, flat = 0;
    Photon p;
    State s;
    int steps = 0, scatter_first = 0;
    uint32_t up_node = 0xFFFFFFFFu;   // the leaf node of the photon's last hit record (walk_up's start)
    uint32_t up_chain = 0xFFFFFFFFu;  // ancestor word `sub` of that node (read during the step's physics)
    uint32_t q = wq ? next_q() : slot, pid = 0, iters = 0, paired_steps = 0;
    bool live = false, exhausted = wq ? q >= n : slot >= nslot;
    unsigned long long t0 = 0, walk_ticks = 0;
    enum { P_WALK, P_PHYS, P_OTHER };
    Prof<3> pf;
    pf.start(P_OTHER);
#ifdef CHR_DEVICE_PROFILE
    LongProf<true> lpf;
#else
    LongProf<false> lpf;
#endif
    // run_photon's write-back (propagate.cu:343-353) and the alive bit
    auto finish = [&]() {
        store3(a.pos, pid, p.pos);
        store3(a.dir, pid, p.dir);
        store3(a.pol, pid, p.pol);
        a.wl[pid] = p.wavelength;
        a.t[pid] = p.time;
        a.flags[pid] = p.history;
        a.last_hit[pid] = p.last_hit;
        a.weights[pid] = p.weight;
        if (sub == 0) {
            if (wq) store_rng(a, q, rng);   // this photon's own slot
            if ((p.history & DEAD_MASK) == 0) atomicOr(a.alive_masks + (q >> 6), 1ull << (q & 63u));
            if (a.diag) {   // the tail's serial chain: longest photon in steps and in time
                const unsigned long long cyc = __builtin_amdgcn_s_memrealtime() - t0;
                atomicMax(a.diag + 1, (uint32_t)steps);
                atomicMax(reinterpret_cast<unsigned long long *>(a.diag + 2),
                          (cyc << 16) | (unsigned long long)(steps > 0xFFFF ? 0xFFFF : steps));
                if (steps > 64) {   // where a long-lived photon's step time goes
                    unsigned long long *d64 = reinterpret_cast<unsigned long long *>(a.diag + 4);
                    atomicAdd(d64, walk_ticks);
                    atomicAdd(d64 + 1, cyc);
                    atomicAdd(d64 + 2, (unsigned long long)iters);
                    atomicAdd(d64 + 3, (unsigned long long)steps);
                    atomicAdd(d64 + 4, 1ull);
                    atomicAdd(d64 + 5, (unsigned long long)paired_steps);
                }
            }
        }
        live = false;
        q = wq ? next_q() : q + cap;
    };
    while (true) {
        if (!live && !exhausted) {   // the slot's next queued photon (dead on entry: skipped, no write-back)
            while (q < n) {
                pid = a.input_queue[q];
                const uint32_t history = a.flags[pid] & 0xFFFFu;   // photon.h:29
                if (history & DEAD_MASK) { q = wq ? next_q() : q + cap; continue; }
                if (wq) load_rng(a, q, rng);
                else if (!have_rng) { load_rng(a, slot, rng); have_rng = true; }
                p.history = history;
                p.pos = load3(a.pos, pid);
                p.dir = load3(a.dir, pid);
                p.dir = p.dir / norm(p.dir);
                p.pol = load3(a.pol, pid);
                p.pol = p.pol / norm(p.pol);
                p.wavelength = a.wl[pid];
                p.time = a.t[pid];
                p.last_hit = a.last_hit[pid];
                p.weight = a.weights[pid];
                steps = 0;
                iters = 0;
                paired_steps = 0;
                up_node = 0xFFFFFFFFu;
                up_chain = 0xFFFFFFFFu;
                walk_ticks = 0;
                scatter_first = a.scatter_first;
                live = true;
                t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
                break;
            }
            if (!live) exhausted = true;
        }
        if (__ballot(live) == 0) break;
        // step head (propagate.cu:279-285 / run_photon)
        bool walk = false;
        if (live) {
            if (steps < a.max_steps) {
                steps++;
                const float prod = ((((p.dir.x * p.dir.y) * p.dir.z) * p.pos.x) * p.pos.y) * p.pos.z;
                if (chr_isnan(prod)) p.history |= CHR_NO_HIT | CHR_NAN_ABORT;
                else walk = true;
            }
            if (!walk) finish();
        }
        // the walk, spread over the wave
        const unsigned long long wm = __ballot(walk && sub == 0);   // bit 8g: group g walks
        lpf.step(walk && sub == 0 && steps > 64);
        int tri = -1;
        float dist = -1.0f;
        const int w = __popcll(wm);
        const unsigned long long tw0 = __builtin_amdgcn_s_memrealtime();
        if (w > 0) {
            pf.tick(P_WALK);   // the whole wave walks
            const int Gs = w == 1 ? 64 : (w == 2 ? 32 : (w <= 4 ? 16 : 8));
            const int si = (int)lane / Gs;
            unsigned long long m = wm;
            for (int i = 0; i < si && m != 0; ++i) m &= m - 1;
            const int src = m != 0 ? __ffsll((long long)m) - 1 : (int)(lane & ~7u);
            const bool act = m != 0;
            V3 o, dd;
            uint32_t last, start = 0xFFFFFFFFu, pre_cur = 0xFFFFFFFFu, pre_push = 0xFFFFFFFFu;
            if (w == 1) {   // one walker: its lane is wave-uniform, scalar reads instead of LDS shuffles
                const int s1 = __ffsll((long long)wm) - 1;
                auto rl = [s1](float x) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), s1)); };
                o = v3(rl(p.pos.x), rl(p.pos.y), rl(p.pos.z));
                dd = v3(rl(p.dir.x), rl(p.dir.y), rl(p.dir.z));
                last = (uint32_t)__builtin_amdgcn_readlane(p.last_hit, s1);
                start = (uint32_t)__builtin_amdgcn_readlane((int)up_node, s1);
                // cursor c > 0 of the climb starts at the start node's c-th ancestor
                const int g0 = s1 & ~7, c = (int)(lane >> 3);
                pre_cur = (uint32_t)__shfl((int)up_chain, g0 + (c > 0 ? c - 1 : 0));
                pre_push = (uint32_t)__builtin_amdgcn_readlane((int)up_chain, g0 + 7);
            } else {
                o = v3(__shfl(p.pos.x, src), __shfl(p.pos.y, src), __shfl(p.pos.z, src));
                dd = v3(__shfl(p.dir.x, src), __shfl(p.dir.y, src), __shfl(p.dir.z, src));
                last = (uint32_t)__shfl(p.last_hit, src);
                start = (uint32_t)__shfl((int)up_node, src);
            }
            const uint32_t seg0 = lane & ~(uint32_t)(Gs - 1);
            float sd;
            uint32_t it;
            // one walker: with an idle wave of the workgroup as its triangle tester when
            // there is one (claimed by the mailbox's PS_IDLE -> PS_POSTING)
            bool paired = false, lost = false;
            // one walker with a previous hit: walk_up from that hit's leaf (ahead of pairing)
            const bool up = Gs == 64 && a.walk_up && start != 0xFFFFFFFFu;
            if (Gs == 64 && !up && a.pair && lds_ld(box + PB_IDLE) != 0u && lds_ld(box + PB_STATE) == PS_IDLE &&
                lds_ld(box + PB_ABORT) == 0u) {
                uint32_t old = PS_TAKEN;
                if (lane == 0) old = atomicCAS(&box_s[PB_STATE], PS_IDLE, PS_POSTING);
                paired = (uint32_t)__builtin_amdgcn_readfirstlane((int)old) == PS_IDLE;
            }
            int st = up ? walk_lone<true>(g, o, dd, last, LdsFlat{wstack}, TAIL_STACK * 8, LdsFlat{wtris}, overflow, sd,
                                          it, __builtin_inff(), 0xFFFFFFFFu, -1, __builtin_inff(),
                                          (start & WIDE_NODE_MASK) | WIDE_CHAIN_MORE, a.walk_up != 4u, pre_cur, pre_push)
                     : paired ? walk_pair(g, top, o, dd, last, LdsFlat{wstack}, TAIL_STACK * 8, wtris,
                                        (threadIdx.x >> 6) * 2u * TAIL_TRI, box, PAIR_SPIN_MAX, overflow, sd, it, lost)
                     : Gs == 64
                         ? walk_lone(g, o, dd, last, LdsFlat{wstack}, TAIL_STACK * 8, LdsFlat{wtris}, overflow, sd, it)
                     : (a.walk_up == 1u || a.walk_up == 4u)   // grouped walks climb from their previous hit's leaf too
                         ? walk_segment<0, LdsFlat, true>(g, act, o, dd, last, Gs,
                                                          LdsFlat{wstack + seg0 / 8 * TAIL_STACK * 2}, TAIL_STACK * Gs / 8,
                                                          LdsFlat{wtris + 4 * seg0}, top, overflow, sd, it,
                                                          __builtin_inff(), 0xFFFFFFFFu, -1, __builtin_inff(),
                                                          start == 0xFFFFFFFFu ? 0u : ((start & WIDE_NODE_MASK) | WIDE_CHAIN_MORE))
                         : walk_segment<0>(g, act, o, dd, last, Gs, LdsFlat{wstack + seg0 / 8 * TAIL_STACK * 2},
                                           TAIL_STACK * Gs / 8, LdsFlat{wtris + 4 * seg0}, top, overflow, sd, it);
            // a lost pair handshake: the tester's minimum may be partial -> the walk again, alone
            if (lost) st = walk_lone(g, o, dd, last, LdsFlat{wstack}, TAIL_STACK * 8, LdsFlat{wtris}, overflow, sd, it);
            if (Gs == 64) {   // one segment: every lane already holds the result
                tri = st;
                dist = sd;
            } else {
                const int mine = __popcll(wm & ((1ull << (lane & ~7u)) - 1ull)) * Gs;   // my group's segment
                tri = __shfl(st, mine);
                dist = __shfl(sd, mine);
                it = (uint32_t)__shfl((int)it, mine);
            }
            if (walk) {
                iters += it;
                paired_steps += paired ? 1u : 0u;
                walk_ticks += __builtin_amdgcn_s_memrealtime() - tw0;
                // the hit record's leaf node (its last word), for the next step's walk_up:
                // in flight during this step's physics
                up_node = tri >= 0 ? gld(reinterpret_cast<const uint32_t *>(g.wtri + 4 * (size_t)tri) + 15) : 0xFFFFFFFFu;
            }
            pf.tick(P_OTHER);
        }
        if (walk) {   // the rest of the step (run_photon's loop body)
            pf.tick(P_PHYS);
            if (sub == 0) {
                pf.call(P_WALK);
                pf.call(P_PHYS);
                const V3 inv = v3(1.0f / p.dir.x, 1.0f / p.dir.y, 1.0f / p.dir.z);
                if (!(chr_isfinite(inv.x) && chr_isfinite(inv.y) && chr_isfinite(inv.z))) flat++;
            }
            lpf.mark(LP_WALK);
            s.distance = dist;
            Watch wt;
            wt.begin(2u, sub == 0 ? pid : 0xFFFFFFFFu, a.pos, q, slot, p.pos, p.dir, p.last_hit);
            finish_fill<true, WIRES>(g, s, p, tri);
            wt.filled(tri, s);
            // the next walk's start node's ancestor chain (walk_lone<true>'s prefetch), in
            // flight during the rest of the physics: one dependent iteration less
            up_chain = up_node != 0xFFFFFFFFu
                           ? gld(reinterpret_cast<const uint32_t *>(g.wnodes + (size_t)g.wstride * (up_node & WIDE_NODE_MASK)) +
                                 24 + sub)
                           : 0xFFFFFFFFu;
            lpf.mark(LP_FILL);
            bool stop = p.last_hit == -1;
            if (!stop) {
                int command = propagate_to_boundary(g, p, s, rng, a.use_weights, scatter_first);
                lpf.mark(LP_TO_BOUNDARY);
                scatter_first = 0;
                if (command == BREAK) {
                    stop = true;
                } else if (command == PASS) {
                    if (s.surface_index != -1) {
                        command = propagate_at_surface(g, p, s, rng, a.use_weights);
                        if (command == BREAK) stop = true;
                    }
                    if (command == PASS) propagate_at_boundary(p, s, rng);
                }
                lpf.mark(LP_AT_BOUNDARY);
            }
            wt.end(p.pos, p.history, p.time);
            pf.tick(P_OTHER);
            if (stop) finish();
        }
    }
    if (!wq && have_rng && sub == 0) store_rng(a, slot, rng);
    if (sub == 0 && overflow) atomicAdd(a.counters, overflow);
    if (sub == 0 && flat && a.diag) atomicAdd(a.diag, flat);
    serve();
#ifdef CHR_DEVICE_PROFILE
    pf.tick(P_OTHER);
    prof_add(CHR_PROF_TAIL_WALK, pf.calls[P_WALK], pf.cyc[P_WALK]);
    prof_add(CHR_PROF_TAIL_PHYSICS, pf.calls[P_PHYS], pf.cyc[P_PHYS]);
    prof_add(CHR_PROF_TAIL_OTHER, 0ull, pf.cyc[P_OTHER]);
    prof_add(CHR_PROF_TAIL_KERNEL, 1ull, pf.total());
    lpf.flush();
#endif
}

// The reference walk's 48-byte triangle records (v0, e1 = v1-v0, e2 = v2-v0,
// e3 = v2-v1; device_geometry.h) from the wide records, which hold every
// triangle once with its float vertices (chr::geometry_ref_nodes, first use).
__global__ __launch_bounds__(BLOCK) void ref_triangles_kernel(const float4 *wtri, uint32_t nwtri, float4 *tri) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= nwtri) return;
    const float4 r0 = wtri[4 * (size_t)i], r1 = wtri[4 * (size_t)i + 1], r2 = wtri[4 * (size_t)i + 2];
    const V3 v0 = v3(r0.x, r0.y, r0.z), v1 = v3(r0.w, r1.x, r1.y), v2 = v3(r1.z, r1.w, r2.x);
    const V3 e1 = v1 - v0, e2 = v2 - v0, e3 = v2 - v1;
    float4 *o = tri + 3 * (size_t)__float_as_uint(r2.y);
    o[0] = make_float4(v0.x, v0.y, v0.z, e1.x);
    o[1] = make_float4(e1.y, e1.z, e2.x, e2.y);
    o[2] = make_float4(e2.z, e3.x, e3.y, e3.z);
}

// ---------------------------------------------------------------- ray binning (trace order)
// The order in which trace_kernel walks the queued rays does not change any
// result (each walk's result is stored at its queue position), so the first
// step's rays are binned by direction cell (a 22-bit radix sort of 2^22
// octahedral cells in Hilbert order; rounds 1-3: 16 bits, 65,536 cells row-major)
// to make the 64 rays of a wave walk the same subtrees: better L1/L2 reuse of nodes.
__device__ __forceinline__ uint32_t octa_cell(V3 d) {   // octahedral map of a unit vector, Hilbert order of 11+11-bit cells
    const float s = fabsf(d.x) + fabsf(d.y) + fabsf(d.z);
    float u = d.x / s, v = d.y / s;
    if (d.z < 0.0f) {
        const float uu = (1.0f - fabsf(v)) * (u < 0.0f ? -1.0f : 1.0f);
        const float vv = (1.0f - fabsf(u)) * (v < 0.0f ? -1.0f : 1.0f);
        u = uu; v = vv;
    }
    uint32_t x = (uint32_t)fminf(fmaxf((u + 1.0f) * 1024.0f, 0.0f), 2047.0f);
    uint32_t y = (uint32_t)fminf(fmaxf((v + 1.0f) * 1024.0f, 0.0f), 2047.0f);
    uint32_t dkey = 0;
    for (uint32_t sq = 1024u; sq > 0u; sq >>= 1) {   // Hilbert order: no jumps between quadrants
        const uint32_t rx = (x & sq) ? 1u : 0u, ry = (y & sq) ? 1u : 0u;
        dkey += sq * sq * ((3u * rx) ^ ry);
        if (ry == 0u) {   // rotate the quadrant
            if (rx == 1u) { x = 2047u - x; y = 2047u - y; }
            const uint32_t t = x; x = y; y = t;
        }
    }
    return dkey;
}
// direction-binning key of a queued photon (0 for a zero / non-finite direction)
__device__ __forceinline__ uint32_t bin_key_of(V3 d) {
    const float l = sqrtf(d.x * d.x + d.y * d.y + d.z * d.z);
    return (l > 0.0f && l < __builtin_inff()) ? octa_cell(v3(d.x / l, d.y / l, d.z / l)) : 0u;
}
__global__ __launch_bounds__(BLOCK) void bin_key_kernel(const float *dir, const uint32_t *queue, uint32_t n,
                                                        uint32_t *keys, uint32_t *vals) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t pid = queue[i];
    keys[i] = bin_key_of(v3(dir[3 * pid], dir[3 * pid + 1], dir[3 * pid + 2]));
    vals[i] = i;
}
// ---------------------------------------------------------------- wavefront split
// A one-step launch (max_steps == 1, every host step above the tail) is split
// in two kernels:
//   trace_kernel  -- the BVH walk of fill_state (mesh.h:45-126) for every live
//                    queued photon, written as (triangle, distance) per queue
//                    position;
//   shade_kernel  -- the rest of the step, unchanged, reading that walk result
//                    instead of walking.
// A photon's walk depends only on its position, direction and last hit, which
// the step does not change before fill_state, so every result is identical.
// The trace kernel holds only the walk state (no photon physics, no RNG): it
// needs fewer registers and less LDS than the fused step kernel, so more waves
// fit per SIMD to hide the dependent node/triangle fetch latency, and it is
// persistent: a lane whose walk ends fetches the next queued photon (wave-batched
// atomic ray counter) instead of idling until the slowest lane of its wave ends.
struct TraceArgs {
    const float *pos, *dir;
    const uint32_t *flags;
    const int32_t *last_hit;
    const uint32_t *queue;       // this step's queue
    uint32_t n;                  // queue length
    int2 *hits;                  // per queue position: (triangle or -1, distance bits)
    uint32_t *next;              // ray counter (zeroed by the host)
    uint32_t *counters;          // [0] overflows, [2..] u64 walk counters (COUNT)
    const uint32_t *order;       // fetch order: the j-th ray walked is queue position order[j] (nullptr: j)
    const uint4 *rays;           // ray records in walk order (2 x uint4 per ray, ray_record; nullptr: gather
                                 // queue -> flags / pos / dir / last_hit per refill instead)
    uint32_t *walk_hist;         // COUNT: [0..31] walks by log2(nodes + triangles), [32..33] u64 max (cost << 32 | photon)
    uint2 *spill;                // stack entries >= SL: (WIDE_STACK - SL) x gridDim.x*BLOCK, entry-major (HBM, no scratch)
    uint32_t *diag;              // [0] += flat rays walked by this launch (nullptr: off)
    // device-driven steps (nullptr: host-driven): the queue length is *dev_n - 1
    // (the input queue's count header) and the launch runs only if *mode is STEP_ONE
    const uint32_t *dev_n;
    const uint32_t *mode;
};
constexpr uint32_t CLAIM = 64;       // rays a wave takes from the ray counter per refill (at most)
constexpr uint32_t DRAIN_MAX = 4;    // a wave drains its last <= DRAIN_MAX walks whole-wave

// Ray record of one queue position, the only thing trace_kernel's refill
// reads: written in walk order by the kernel that builds the queue (the
// previous step's scatter, or the first step's classification + permutation),
// so a refill is one 32-byte load, contiguous across the refilling lanes,
// instead of the dependent order -> queue -> flags / pos / dir / last_hit chain
// of the photon arrays (propagate.cu:280-293).  Words: origin, the normalised
// direction (propagate.cu:280-281, the same float operations as the walk
// made), the photon's last hit, its queue position; bit 31 of the last word:
// no walk here (dead on entry, or NaN state).
constexpr uint32_t RAY_SKIP = 0x80000000u;
__device__ __forceinline__ void put_ray(uint4 *rays, uint32_t j, V3 o, V3 d, int32_t last_hit, uint32_t q, bool walk) {
    rays[2 * (size_t)j] = make_uint4(__float_as_uint(o.x), __float_as_uint(o.y), __float_as_uint(o.z),
                                     __float_as_uint(d.x));
    rays[2 * (size_t)j + 1] = make_uint4(__float_as_uint(d.y), __float_as_uint(d.z), (uint32_t)last_hit,
                                         q | (walk ? 0u : RAY_SKIP));
}

// The ray record of photon pid at queue position p, written at walk position j.
__device__ __forceinline__ void put_photon_ray(const float *pos, const float *dir, uint32_t pid, uint32_t p,
                                               uint4 *rays, const int32_t *last_hit, uint32_t j) {
    const V3 o = load3(pos, pid);
    V3 d = load3(dir, pid);
    d = d / norm(d);
    put_ray(rays, j, o, d, last_hit[pid], p, walk_kind(o, d) == 1);
}

// first host step: with keys, the direction-binning key of every queue
// position (bin_key_kernel's, one pass over the photons instead of two), and
// with rays the ray record of every queue position at its own index (binned:
// permuted into walk order after the sort)
__global__ __launch_bounds__(BLOCK) void classify_kernel(const float *pos, const float *dir, const uint32_t *flags,
                                                         const int32_t *last_hit, const uint32_t *queue, uint32_t n,
                                                         uint32_t *keys, uint32_t *vals, uint4 *rays) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t pid = queue[i];
    if (keys) {
        keys[i] = bin_key_of(v3(dir[3 * pid], dir[3 * pid + 1], dir[3 * pid + 2]));
        vals[i] = i;
    }
    if ((flags[pid] & 0xFFFFu) & DEAD_MASK) {
        if (rays) put_ray(rays, i, v3(0.0f, 0.0f, 0.0f), v3(0.0f, 0.0f, 0.0f), -1, i, false);
        return;
    }
    if (rays) put_photon_ray(pos, dir, pid, i, rays, last_hit, i);
}

// rays_out[j] = rays_in[order[j]]: the first step's records in the binned walk order
__global__ __launch_bounds__(BLOCK) void permute_rays_kernel(const uint4 *rays_in, const uint32_t *order, uint32_t n,
                                                             uint4 *rays_out) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= n) return;
    const uint32_t q = order[j];
    const uint4 r0 = rays_in[2 * (size_t)q], r1 = rays_in[2 * (size_t)q + 1];
    rays_out[2 * (size_t)j] = r0;
    rays_out[2 * (size_t)j + 1] = r1;
}

// COUNT: walk counters; F: triangle step once F/8 of the walking lanes have
// parked leaves (intersect_wide_spec); SL: stack entries in LDS; MINW: waves
// per SIMD; R: refill once R of the 64 lanes are without a ray.
// GATHER: refill from the photon arrays (order -> queue -> flags / pos / dir /
// last hit) instead of the ray records; a separate instantiation, so the
// ray-record kernel's walk loop carries no code of the other refill.
template <bool COUNT, int F, int SL, int MINW, int R, bool GATHER = false>
__global__ __launch_bounds__(BLOCK, MINW) void trace_kernel(const DevGeom *__restrict__ gdev, TraceArgs a) {
    constexpr int TB = BLOCK;
    __shared__ uint32_t lds[(2 * SL + LEAFQ) * TB];
    // a draining wave's walk_segment stacks (8 x DSTK entries, DSTK per 8 lanes) + triangle
    // lists in its LDS rows
    constexpr int DSTK = ((2 * SL + LEAFQ) * 64 - 2 * TAIL_TRI) / 16;
    // a walk's stack holds >= 112 entries: 16 lanes per walk (<= DRAIN_MAX = 4 walks) need 2 * DSTK
    static_assert(2 * DSTK >= 112, "drain needs the wave's LDS rows");
    WStack st;
    // Deep stack entries live in a lane-strided HBM column sized for this
    // persistent grid, not in private scratch: a kernel with a private segment
    // depends on the runtime's scratch allocation, which can throttle the waves
    // a dispatch keeps resident (the persistent grid then drains on a few waves).
    st.spill = a.spill + (blockIdx.x * TB + threadIdx.x);
    st.sstride = gridDim.x * TB;
    st.node = (CHR_LDS uint32_t *)(lds + threadIdx.x);
    st.dist = (CHR_LDS float *)(lds + SL * TB + threadIdx.x);
    st.leafq = (CHR_LDS uint32_t *)(lds + 2 * SL * TB + threadIdx.x);
    if (a.mode && *a.mode != STEP_ONE) return;
    const uint32_t n = a.dev_n ? *a.dev_n - 1u : a.n;
    const DevGeom &g = *gdev;
    const TopNodes top{nullptr, 0u};
    const uint32_t lane = __lane_id();
    uint32_t overflow = 0;
    WalkCounts cnt{0u, 0u, 0u, 0u, 0u, 0ull, 0ull, 0u};
    bool has_ray = false, exhausted = false;
    uint32_t q = 0, pid = 0, walk_cost = 0;
    const uint32_t total = n;       // work items: the queued rays
    uint32_t nflat_rays = 0;        // flat rays walked by this work-item (flat-axis slab test; diagnostic)
    V3 o = v3(0.0f, 0.0f, 0.0f), d = v3(0.0f, 0.0f, 1.0f);
    RaySlab slab = make_slab(o, o, d);
    float best = 0.0f, best_bd = 0.0f, cut = 0.0f;   // best hit, its leaf box's entry, the culling threshold
    uint32_t best_rank = 0, last = 0, node = 0;
    int best_id = -1, sp = 0;
    bool walk_done = true, drain = false;
    uint32_t qh = 0, qt = 0, pcur = 0, pleft = 0;
    constexpr uint32_t INVALID = 0xFFFFFFFFu;
    // claim size: CLAIM, or a wave's share of a launch smaller than the grid's lanes
    // (every wave then walks a few rays and reaches its drain sooner; r03 ab24/ab25:
    // trace 14.40 -> 14.32 ms per step, the last launches 0.39 -> 0.37 ms)
    uint32_t claim = CLAIM;
    {
        const uint32_t waves = gridDim.x * (TB / 64);
        const uint32_t share = (total + waves - 1u) / waves;
        claim = share < 1u ? 1u : (share < CLAIM ? share : CLAIM);
    }
    enum { P_NODE, P_TRI, P_REFILL, P_IDLE, P_DRAIN, P_BOX = 3 };   // regions (calls: P_REFILL = walks, P_BOX = boxes)
    Prof<5> pf;
    pf.start(P_REFILL);
#ifdef CHR_DEVICE_PROFILE
    bool wlog = false;   // this lane walks the watched ray
#endif
    while (true) {
        pf.tick(P_REFILL);   // the last step goes to the region each work-item was in
        if (has_ray && walk_done && pleft == 0 && qh == qt) {   // walk over: publish (mesh.h:123-125)
            CHR_WEV(wlog, 9u, q, (uint32_t)best_id, __float_as_uint(best), best_rank, 0u, 0u, 0u);
            a.hits[q] = make_int2(best_id, __float_as_int(best_id == -1 ? -1.0f : best));
            has_ray = false;
            if constexpr (COUNT) {
                if (a.walk_hist) {
                    atomicAdd(a.walk_hist + (31 - __builtin_clz(walk_cost + 1)), 1u);
                    atomicMax(reinterpret_cast<unsigned long long *>(a.walk_hist + 32),
                              ((unsigned long long)walk_cost << 32) | pid);
                }
            }
        }
        if (!exhausted) {
            const unsigned long long need = __ballot(!has_ray);
            if (need != 0 && (__popcll(need) >= R || need == __ballot(1))) {
                const uint32_t want = (uint32_t)__popcll(need) < claim ? (uint32_t)__popcll(need) : claim;
                const uint32_t rank = (uint32_t)__popcll(need & ((1ull << lane) - 1ull));
                const int leader = __ffsll((long long)need) - 1;
                uint32_t base = 0;
                if ((int)lane == leader) base = atomicAdd(a.next, want);
                base = __shfl(base, leader);
                if (base + want >= total) exhausted = true;
                const uint32_t j = base + rank;
                if (!has_ray && rank < want) {
                    bool start = false;
                    if (!GATHER && j < n) {
                        // the ray record: one 32-B load (put_ray); skip bit: dead / NaN
                        const uint4 r0 = gld(a.rays + 2 * (size_t)j), r1 = gld(a.rays + 2 * (size_t)j + 1);
                        q = r1.w & ~RAY_SKIP;
                        if (!(r1.w & RAY_SKIP)) {
                            o = v3(__uint_as_float(r0.x), __uint_as_float(r0.y), __uint_as_float(r0.z));
                            d = v3(__uint_as_float(r0.w), __uint_as_float(r1.x), __uint_as_float(r1.y));
                            last = r1.z;
                            if constexpr (COUNT) pid = a.walk_hist ? a.queue[q] : q;
                            start = true;
                            node = 0;
                            best = __builtin_inff();
                            best_bd = __builtin_inff();
                            cut = __builtin_inff();
                            best_rank = 0xFFFFFFFFu;
                        }
                    } else if (GATHER && j < n) {
                        q = a.order ? a.order[j] : j;
                        pid = a.queue[q];
                        // dead on entry / NaN: no walk (the step kernel skips / aborts them)
                        if (!((a.flags[pid] & 0xFFFFu) & DEAD_MASK)) {
                            o = load3(a.pos, pid);
                            d = load3(a.dir, pid);
                            d = d / norm(d);                        // propagate.cu:280-281
                            if (walk_kind(o, d) == 1) {
                                start = true;
                                node = 0;
                                best = __builtin_inff();
                                best_bd = __builtin_inff();
                                cut = __builtin_inff();
                                best_rank = 0xFFFFFFFFu;
                                last = (uint32_t)a.last_hit[pid];
                            }
                        }
                    }
                    if (start) {
                        slab = make_slab(o, v3(-o.x / d.x, -o.y / d.y, -o.z / d.z), v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z));
                        best_id = -1;
                        sp = 0;
                        walk_done = false;
                        has_ray = true;
                        walk_cost = 0;
                        pf.call(P_REFILL);
                        if (slab.flat) nflat_rays++;
                        if constexpr (COUNT) cnt.walks++;
#ifdef CHR_DEVICE_PROFILE
                        wlog = wray_match(o);
                        CHR_WEV(wlog, 1u, q, j, blockIdx.x, threadIdx.x, __float_as_uint(d.x), __float_as_uint(d.y),
                                __float_as_uint(d.z));
#endif
                    }
                }
            }
        }
        if constexpr (!COUNT) {
            // Drain: once the ray counter is exhausted and at most 8 ordinary walks
            // are left in the wave, the whole wave finishes them together
            // (walk_segment: 8..64 lanes per walk, Gs/8 cursors each, a dependent
            // step's triangles in parallel) instead of one lane each.  The last
            // walks of a launch are its longest (~200 node + triangle steps at
            // ~2 us per dependent step on the 29k detector: the 0.4 ms floor of
            // every small launch).  Each restarts from the root seeded with its
            // best so far (conservative culling, the same nearest hit); the
            // lanes' stacks are abandoned and their LDS rows reused.
            if (exhausted && __ballot(has_ray) != 0 && (uint32_t)__popcll(__ballot(has_ray)) <= DRAIN_MAX) {
                drain = true;   // after the loop, where the walk state below is no longer live
                break;
            }
        }
        pf.tick(P_IDLE);
        const bool has_work = has_ray && (pleft != 0 || qh != qt);
        const bool can_walk = has_ray && !walk_done && (qt - qh) <= (uint32_t)(LEAFQ - 8);
        const unsigned long long mw = __ballot(can_walk);
        const unsigned long long mt = __ballot(has_work);
        if ((mw | mt) == 0) {
            if (exhausted && __ballot(has_ray) == 0) {
                break;
            }
            continue;                                    // walks ended: publish + refill
        }
        if (mw != 0 && 8 * __popcll(mt) < F * __popcll(mw | mt)) {
            // ------------------------------------------------ node step
            if (!can_walk) continue;
            pf.set(P_NODE);
            if (node == INVALID) {
                bool found = false;
                while (sp > 0) {
                    sp--;
                    float t;
                    wpop<SL, TB>(st, sp, node, t);
                    CHR_WEV(wlog, 2u, node, __float_as_uint(t), __float_as_uint(best), (uint32_t)sp, 0u, 0u, 0u);
                    if (!(t > cut)) { found = true; break; }
                }
                if (!found) { walk_done = true; continue; }
            }
            if constexpr (COUNT) { cnt.nodes++; walk_cost++; if (wave_leader()) cnt.wave_nodes++; }
            uint4 h, a1, a2, a3, a4, a5;
            {
                const uint4 *np = g.wnodes + (size_t)g.wstride * node;
                h = gld(np); a1 = gld(np + 1); a2 = gld(np + 2); a3 = gld(np + 3); a4 = gld(np + 4); a5 = gld(np + 5);
            }
#ifdef CHR_DEVICE_PROFILE
            pf.call(P_NODE);
            for (int k = 0; k < 8; ++k)
                pf.call(P_BOX, (((k < 4 ? a4.z : a4.w) >> (8 * (k & 3))) & 0xFFu) != 0u ? 1u : 0u);
#endif
            uint32_t near_node;
            float near_t;
            uint32_t leaf_mask =
                expand_node<SL, TB>(h, a1, a2, a3, a4, a5, slab, cut, near_node, near_t, st, sp, overflow, 0xFFu);
            CHR_WEV(wlog, 3u, node, near_node, __float_as_uint(near_t), leaf_mask, (uint32_t)sp, __float_as_uint(best),
                    qt - qh);
            node = near_node;
            while (leaf_mask) {
                const int k = __builtin_ctz(leaf_mask);
                leaf_mask &= leaf_mask - 1;
                const uint32_t kind = ((k < 4 ? a4.z : a4.w) >> (8 * (k & 3))) & 0xFFu;
                const uint32_t first = a4.y + (((k < 4 ? a5.x : a5.y) >> (8 * (k & 3))) & 0xFFu);
                st.leafq[(qt % LEAFQ) * TB] = first | ((kind - 1u) << 30);
                qt++;
            }
        } else {
            // ------------------------------------------------ triangle step
            if (!has_work) continue;
            pf.set(P_TRI);
            pf.call(P_TRI);
            if (pleft == 0) {
                const uint32_t e = st.leafq[(qh % LEAFQ) * TB];
                qh++;
                pcur = e & 0x3FFFFFFFu;
                pleft = (e >> 30) + 1u;
            }
            if constexpr (COUNT) { cnt.tris++; walk_cost++; if (wave_leader()) cnt.wave_tris++; }
            const float4 *r = g.wtri + 4 * (size_t)pcur;
            const float4 r0 = gld(r), r1 = gld(r + 1), r2 = gld(r + 2);
            pcur++;
            pleft--;
            const uint32_t id = __float_as_uint(r2.y);
            float dist;
            CHR_WEV(wlog, 4u, (uint32_t)rec_of(g, r), id, __float_as_uint(best), pleft, 0u, 0u, 0u);
            if (id == last ||
                !intersect_record(o, d, r0, r1, r2, dist))
                continue;
            const uint32_t rank = __float_as_uint(r2.z);
            CHR_WEV(wlog, 5u, (uint32_t)rec_of(g, r), id, __float_as_uint(dist), rank, __float_as_uint(best), best_rank, 0u);
            if (!ref_may_beat(dist, rank, best, best_rank, best_bd)) continue;
            const float4 r3 = gld(r + 3);
            V3 lo, hi;
            node_bounds(g, make_uint4(__float_as_uint(r2.w), __float_as_uint(r3.x), __float_as_uint(r3.y), 0u), lo, hi);
            float bd;
            const bool boxok = intersect_box_slab(slab, lo, hi, bd);
            CHR_WEV(wlog, 6u, (uint32_t)rec_of(g, r), id, boxok ? 1u : 0u, __float_as_uint(bd), __float_as_uint(best), 0u, 0u);
            if (!boxok || !ref_beats(dist, rank, bd, best, best_rank, best_bd)) continue;   // mesh.h:94-96
            best = dist;
            best_bd = bd;
            cut = ref_cut(best, best_bd);
            best_rank = rank;
            best_id = rec_of(g, r);
        }
    }
    if constexpr (!COUNT) {
        if (drain) {
            pf.tick(P_DRAIN);
            CHR_WEV(wlog && has_ray, 7u, q, (uint32_t)best_id, __float_as_uint(best), best_rank, (uint32_t)__popcll(__ballot(has_ray)),
                    0u, 0u);
            const unsigned long long rm = __ballot(has_ray);
            const int w = __popcll(rm);
            const int Gs = w == 1 ? 64 : (w == 2 ? 32 : 16);
            const int si = (int)lane / Gs;
            unsigned long long m = rm;
            for (int i = 0; i < si && m != 0; ++i) m &= m - 1;
            const bool act = m != 0;
            const int src = act ? __ffsll((long long)m) - 1 : (int)lane;
            const V3 so = v3(__shfl(o.x, src), __shfl(o.y, src), __shfl(o.z, src));
            const V3 sdir = v3(__shfl(d.x, src), __shfl(d.y, src), __shfl(d.z, src));
            const uint32_t slast = (uint32_t)__shfl((int)last, src);
            const float sbest = __shfl(best, src), sbd = __shfl(best_bd, src);
            const uint32_t srank = (uint32_t)__shfl((int)best_rank, src);
            const int sid = __shfl(best_id, src);
            const int seg0 = (int)lane & ~(Gs - 1);
            CHR_LDS uint32_t *wbase = (CHR_LDS uint32_t *)(lds + (threadIdx.x & ~63u));
            float sdist;
            uint32_t sit;
            const int tri = w == 1
                                ? walk_lone(g, so, sdir, slast, LdsRowsT<TB>{wbase, 0}, DSTK * 8,
                                            LdsRowsT<TB>{wbase, 8 * DSTK * 2}, overflow, sdist, sit, sbest, srank, sid, sbd)
                                : walk_segment<0>(g, act, so, sdir, slast, Gs, LdsRowsT<TB>{wbase, seg0 / 8 * DSTK * 2},
                                                  DSTK * Gs / 8, LdsRowsT<TB>{wbase, 8 * DSTK * 2 + 4 * seg0}, top,
                                                  overflow, sdist, sit, sbest, srank, sid, sbd);
            const int mine = (__popcll(rm & ((1ull << lane) - 1ull)) * Gs) & 63;   // my segment's first lane
            const int rt = __shfl(tri, mine);
            const float rd = __shfl(sdist, mine);
            if (has_ray) {                                        // publish (mesh.h:123-125)
                CHR_WEV(wlog, 8u, q, (uint32_t)rt, __float_as_uint(rd), 0u, 0u, 0u, 0u);
                a.hits[q] = make_int2(rt, __float_as_int(rt == -1 ? -1.0f : rd));
                pf.call(P_DRAIN);
            }
            pf.tick(P_IDLE);
        }
    }
#ifdef CHR_DEVICE_PROFILE
    pf.tick(P_IDLE);
    prof_add(CHR_PROF_INTERSECT_MESH, pf.calls[P_REFILL], (unsigned long long)pf.cyc[P_NODE] + pf.cyc[P_TRI]);
    prof_add(CHR_PROF_INTERSECT_NODE, pf.calls[P_NODE], pf.cyc[P_NODE]);
    prof_add(CHR_PROF_INTERSECT_TRIANGLE, pf.calls[P_TRI], pf.cyc[P_TRI]);
    prof_add(CHR_PROF_INTERSECT_BOX, pf.calls[P_BOX], 0ull);
    prof_add(CHR_PROF_TRACE_REFILL, 0ull, pf.cyc[P_REFILL]);
    prof_add(CHR_PROF_TRACE_IDLE, 0ull, pf.cyc[P_IDLE]);
    prof_add(CHR_PROF_TRACE_DRAIN, pf.calls[P_DRAIN], pf.cyc[P_DRAIN]);
    prof_add(CHR_PROF_TRACE_KERNEL, 1ull, pf.total());
#endif
    if (overflow) atomicAdd(a.counters, overflow);
    if (a.diag && nflat_rays) atomicAdd(a.diag, nflat_rays);
    if constexpr (COUNT) {
        unsigned long long *c64 = reinterpret_cast<unsigned long long *>(a.counters + 2);
        atomicAdd(c64, (unsigned long long)cnt.nodes);
        atomicAdd(c64 + 1, (unsigned long long)cnt.tris);
        atomicAdd(c64 + 2, (unsigned long long)cnt.walks);
        atomicAdd(c64 + 3, (unsigned long long)cnt.wave_nodes);
        atomicAdd(c64 + 4, (unsigned long long)cnt.wave_tris);
    }
}

// Two-level exclusive scan of the popcounts of nwords alive/selection masks.
// mask_block_scan_kernel: workgroup b scans words [256b, 256b+256) -> word_offsets
// (exclusive within the workgroup) and block_sums[b]; scan_block_sums_kernel
// (one workgroup) turns block_sums into exclusive block prefixes, records
// base[0] = out_counter[0] on entry, out_counter[0] += total, total_out = total.
// Consumers add block_prefix[w >> 8] to word_offsets[w].
constexpr int SCAN_WORDS = 256;
__global__ __launch_bounds__(SCAN_WORDS) void mask_block_scan_kernel(const unsigned long long *masks, uint32_t nwords,
                                                                     uint32_t *word_offsets, uint32_t *block_sums,
                                                                     const uint32_t *dev_n, const uint32_t *mode,
                                                                     uint32_t skip) {
    __shared__ uint32_t wave_tot[SCAN_WORDS / 64];
    if (mode && (*mode == STEP_IDLE || *mode == skip)) return;
    if (dev_n) nwords = (*dev_n - 1u + 63u) / 64u;
    const uint32_t w = blockIdx.x * SCAN_WORDS + threadIdx.x;
    const uint32_t c = w < nwords ? (uint32_t)__popcll(masks[w]) : 0u;
    // inclusive scan within the wave (shuffles), then across the 4 waves
    uint32_t x = c;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    const int wid = threadIdx.x >> 6;
    if (lane == 63) wave_tot[wid] = x;
    __syncthreads();
    uint32_t before = 0;
    for (int k = 0; k < wid; ++k) before += wave_tot[k];
    if (w < nwords) word_offsets[w] = before + x - c;
    if (threadIdx.x == SCAN_WORDS - 1) block_sums[blockIdx.x] = before + x;
}

// The head of a device-driven step slot (step_head_kernel, or folded into the
// previous slot's scan_block_sums_kernel): the queue length n picks the slot's
// mode -- the nsteps policy of photon.py:261-264 (one-step launch; the multi-step
// tail below `tail_below` photons or with use_weights, when more than one step
// remains; nothing once the queue is empty or the tail ran) -- and resets the
// trace ray counter.  Returns the mode.
struct HeadNext {                      // the next slot's head words (mode == nullptr: no fold)
    uint32_t *mode, *n_out, *done, *ray_counter, *host_ring;
    uint32_t tail_below, max_n;
    int32_t remaining, use_weights;
};
__device__ __forceinline__ uint32_t slot_head(uint32_t n, const HeadNext &h) {
    uint32_t m = STEP_IDLE;
    if (!h.done[0]) {
        if (n == 0 || n > h.max_n) h.done[0] = 1u;   // empty (or a corrupt header: run nothing)
        else if ((n < h.tail_below || h.use_weights) && h.remaining > 1) { m = STEP_TAIL; h.done[0] = 1u; }
        else m = STEP_ONE;
    }
    h.mode[0] = m;
    h.n_out[0] = n;
    // the host's copy of (mode, length), in pinned host memory: read once the
    // slot's trace-start event (ev[2] of device_slots, recorded after this head)
    // has completed (no copy dispatch per slot)
    if (h.host_ring) { h.host_ring[0] = m; h.host_ring[1] = n; }
    if (m != STEP_IDLE) h.ray_counter[0] = 0u;
    return m;
}

// fresh: the output queue starts empty (device-driven slots: base 1, header 1 + total,
// no reset of the header needed); hn: the next slot's head, folded in (one dispatch
// fewer per slot) -- run even when this slot's scan is skipped (its mode then IDLE)
__global__ __launch_bounds__(1024) void scan_block_sums_kernel(uint32_t *block_sums, uint32_t nblocks,
                                                               uint32_t *out_counter, uint32_t *base,
                                                               uint32_t *total_out, const uint32_t *mode,
                                                               uint32_t skip, uint32_t fresh, HeadNext hn) {
    __shared__ uint32_t partial[1024];
    if (mode && (*mode == STEP_IDLE || *mode == skip)) {
        if (hn.mode && threadIdx.x == 0) slot_head(0u, hn);
        return;
    }
    const uint32_t tid = threadIdx.x;
    const uint32_t per = (nblocks + 1023) / 1024;
    const uint32_t b0 = tid * per;
    uint32_t sum = 0;
    for (uint32_t k = 0; k < per && b0 + k < nblocks; ++k) sum += block_sums[b0 + k];
    partial[tid] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = (tid >= off) ? partial[tid - off] : 0;
        __syncthreads();
        partial[tid] += v;
        __syncthreads();
    }
    uint32_t run = partial[tid] - sum;
    for (uint32_t k = 0; k < per && b0 + k < nblocks; ++k) {
        const uint32_t v = block_sums[b0 + k];
        block_sums[b0 + k] = run;
        run += v;
    }
    if (tid == 1023) {
        const uint32_t total = partial[1023];
        if (fresh) {
            if (base) base[0] = 1u;
            if (out_counter) out_counter[0] = 1u + total;
        } else {
            if (base) base[0] = out_counter ? out_counter[0] : 0u;
            if (out_counter) out_counter[0] += total;
        }
        if (total_out) total_out[0] = total;
        if (hn.mode) slot_head(total, hn);   // the next slot's queue is this slot's survivors
    }
}

__device__ __forceinline__ uint32_t word_offset(const uint32_t *word_offsets, const uint32_t *block_prefix, uint32_t w) {
    return word_offsets[w] + block_prefix[w / SCAN_WORDS];
}

// Survivors of a split step also write their next walk's ray record
// (RayEnrol: the next step's records, in queue order; pos == nullptr: off).
struct RayEnrol {
    const float *pos, *dir;
    uint4 *rays;
    const int32_t *last_hit;
};
__global__ __launch_bounds__(BLOCK) void scatter_queue_kernel(const unsigned long long *masks, const uint32_t *word_offsets,
                                                               const uint32_t *block_prefix, const uint32_t *base,
                                                               const uint32_t *in_queue, int32_t first, int32_t n,
                                                               uint32_t *out_queue, RayEnrol fe, const uint32_t *dev_n,
                                                               const uint32_t *mode, uint32_t skip) {
    // skip: a second mode that runs nothing here (a tail run on its own stream
    // by chr_propagate_batches leaves no queue behind)
    if (mode && (*mode == STEP_IDLE || *mode == skip)) return;
    if (dev_n) n = (int32_t)(*dev_n - 1u);
    // grid-stride (device-driven steps launch one grid for any queue length)
    for (int id = blockIdx.x * BLOCK + threadIdx.x; id < n; id += gridDim.x * BLOCK) {
        const unsigned long long m = masks[id >> 6];
        const int lane = id & 63;
        if ((m >> lane) & 1ull) {
            const uint32_t rank = __popcll(m & ((1ull << lane) - 1ull));
            const uint32_t o = base[0] + word_offset(word_offsets, block_prefix, (uint32_t)id >> 6) + rank;
            const uint32_t pid = in_queue[first + id];
            out_queue[o] = pid;
            // out_queue[0] is the count header: position o - 1 of the next step's queue
            if (fe.pos) put_photon_ray(fe.pos, fe.dir, pid, o - 1u, fe.rays, fe.last_hit, o - 1u);
        }
    }
}

// Head of a device-driven step slot: the input queue's length picks the slot's
// mode -- the nsteps policy of photon.py:261-264 (one-step launch; the
// multi-step tail below `tail_below` photons or with use_weights, when more
// than one step remains; nothing once the queue is empty or the tail ran) --
// and the slot's bookkeeping is reset: output queue header, trace ray counter.
__global__ void step_head_kernel(const uint32_t *in_hdr, uint32_t *out_hdr, uint32_t *mode, uint32_t *n_out,
                                 uint32_t *done, uint32_t *ray_counter, uint32_t tail_below, int32_t remaining,
                                 int32_t use_weights, uint32_t max_n, uint32_t *host_ring) {
    if (threadIdx.x != 0) return;
    const HeadNext h{mode, n_out, done, ray_counter, host_ring, tail_below, max_n, remaining, use_weights};
    if (slot_head(in_hdr[0] - 1u, h) != STEP_IDLE) out_hdr[0] = 1u;
}

// alive-mask words of a tail slot (OR-ed by its kernel) zeroed, for the slot's queue length
constexpr uint32_t kClearBlocks = 4;
__global__ __launch_bounds__(BLOCK) void clear_masks_kernel(unsigned long long *masks, const uint32_t *dev_n,
                                                            const uint32_t *mode) {
    if (*mode != STEP_TAIL) return;
    const uint32_t nwords = (*dev_n - 1u + 63u) / 64u;
    for (uint32_t w = blockIdx.x * BLOCK + threadIdx.x; w < nwords; w += gridDim.x * BLOCK) masks[w] = 0ull;
}

// photon.py:242-250: input queue entries (from q0[1]) = photon ids with the
// ncopies clones of a photon interleaved; count headers q0[0] = n + 1 (the
// input's length, read by device-driven steps), q1[0] = 1 (empty output).
// The first block also zeroes the propagate's small control regions (step
// counters, flat-walk control words, the slot loop's done flag): one launch
// instead of a fill dispatch each.
struct ZeroWords {
    uint32_t *p[3];
    uint32_t n[3];   // words (<= BLOCK each)
};
__global__ __launch_bounds__(BLOCK) void init_queue_kernel(uint32_t *q0, uint32_t *q1, uint32_t n, uint32_t true_n,
                                                           uint32_t ncopies, ZeroWords z) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (blockIdx.x == 0)
        for (int k = 0; k < 3; ++k)
            if (z.p[k] && threadIdx.x < z.n[k]) z.p[k][threadIdx.x] = 0u;
    if (i >= n) return;
    q0[1 + i] = i / ncopies + (i % ncopies) * true_n;
    if (i == 0) { q0[0] = n + 1u; q1[0] = 1u; }
}

// ---------------------------------------------------------------- RNG init
__global__ __launch_bounds__(BLOCK) void init_rng_kernel(uint32_t *states, uint32_t nslots, unsigned long long seed,
                                                          unsigned long long subseq0, unsigned long long offset,
                                                          const uint32_t *seq, int nseq, const uint32_t *off, int noff) {
    const uint32_t s = blockIdx.x * BLOCK + threadIdx.x;
    if (s >= nslots) return;
    chr_xorwow r;
    chr_xorwow_init(&r, seed, subseq0 + s, offset, seq, nseq, off, noff);
    states[s] = r.d; states[nslots + s] = r.v0; states[2 * nslots + s] = r.v1;
    states[3 * nslots + s] = r.v2; states[4 * nslots + s] = r.v3; states[5 * nslots + s] = r.v4;
}

// ---------------------------------------------------------------- selection kernels
struct PhotonPtrs {
    float *pos, *dir, *pol, *wl, *t, *weights;
    uint32_t *flags;
    int32_t *last_hit;
    uint32_t *evidx;
};

__device__ __forceinline__ void copy_photon(const PhotonPtrs &src, uint32_t i, const PhotonPtrs &dst, uint32_t o) {
    store3(dst.pos, o, load3(src.pos, i));
    store3(dst.dir, o, load3(src.dir, i));
    store3(dst.pol, o, load3(src.pol, i));
    dst.wl[o] = src.wl[i];
    dst.t[o] = src.t[i];
    dst.flags[o] = src.flags[i];
    dst.last_hit[o] = src.last_hit[i];
    dst.weights[o] = src.weights[i];
    dst.evidx[o] = src.evidx[i];
}

// mode 0: hits (count_photon_hits, propagate.cu:172-199); mode 1: flag select (count_photons, 70-95)
__global__ __launch_bounds__(BLOCK) void flag_kernel(PhotonPtrs ph, int32_t start, int32_t n, uint32_t state,
                                                      const uint32_t *solid_map, const int32_t *solid_to_channel,
                                                      int mode, unsigned long long *masks) {
    const int id = blockIdx.x * BLOCK + threadIdx.x;
    unsigned hit = 0;
    if (id < n) {
        const uint32_t i = (uint32_t)(start + id);
        if (ph.flags[i] & state) {
            if (mode == 1) hit = 1;
            else {
                const int tri = ph.last_hit[i];
                if (tri > -1) hit = solid_to_channel[solid_map[tri]] >= 0;
            }
        }
    }
    const unsigned long long m = __ballot(hit);
    if ((threadIdx.x & 63) == 0 && id < n) masks[id >> 6] = m;
}

__global__ __launch_bounds__(BLOCK) void copy_selected_kernel(PhotonPtrs ph, int32_t start, int32_t n,
                                                               const unsigned long long *masks,
                                                               const uint32_t *word_offsets,
                                                               const uint32_t *block_prefix, PhotonPtrs out,
                                                               int32_t *channels, const uint32_t *solid_map,
                                                               const int32_t *solid_to_channel) {
    const int id = blockIdx.x * BLOCK + threadIdx.x;
    if (id >= n) return;
    const unsigned long long m = masks[id >> 6];
    const int lane = id & 63;
    if (!((m >> lane) & 1ull)) return;
    const uint32_t o = word_offset(word_offsets, block_prefix, (uint32_t)id >> 6) + __popcll(m & ((1ull << lane) - 1ull));
    const uint32_t i = (uint32_t)(start + id);
    copy_photon(ph, i, out, o);
    if (channels) channels[o] = solid_to_channel[solid_map[ph.last_hit[i]]];
}

// propagate.cu:141-169
__global__ __launch_bounds__(BLOCK) void copy_queue_kernel(PhotonPtrs ph, int32_t first, int32_t n, const uint32_t *queue,
                                                            PhotonPtrs out) {
    const int id = blockIdx.x * BLOCK + threadIdx.x;
    if (id >= n) return;
    const uint32_t o = (uint32_t)(first + id);
    copy_photon(ph, queue[o], out, o);
}

// propagate.cu:29-68
__global__ __launch_bounds__(BLOCK) void duplicate_kernel(PhotonPtrs ph, int32_t first, int32_t n, int32_t copies,
                                                           int32_t stride) {
    const int id = blockIdx.x * BLOCK + threadIdx.x;
    if (id >= n) return;
    const uint32_t i = (uint32_t)(first + id);
    for (int c = 1; c <= copies; ++c) copy_photon(ph, i, ph, i + (uint32_t)(stride * c));
}

// mesh.h:131-159
template <bool WIDE>
__global__ __launch_bounds__(BLOCK) void distance_kernel(const DevGeom *__restrict__ gdev, uint32_t n, const float *origin, const float *dir,
                                                          float *distance, uint32_t *counters) {
    __shared__ uint32_t lds_stack[WIDE ? lds_words(WIDE) * BLOCK : STACK_LDS * BLOCK];
    const uint32_t id = blockIdx.x * BLOCK + threadIdx.x;
    if (id >= n) return;
    const DevGeom &g = *gdev;
    V3 o = load3(origin, id), d = load3(dir, id);
    d = d / norm(d);
    uint32_t overflow = 0;
    float dist;
    int tri;
    if constexpr (WIDE) {
        WStack st;
        uint2 wspill[WIDE_STACK - WIDE_LDS];
        st.spill = wspill;
        st.sstride = 1;
        st.node = (CHR_LDS uint32_t *)(lds_stack + threadIdx.x);
        st.dist = (CHR_LDS float *)(lds_stack + WIDE_LDS * BLOCK + threadIdx.x);
        st.leafq = nullptr;
        WalkCounts cnt;
        tri = intersect_wide_sched<false, 2>(g, o, d, dist, -1, st, overflow, cnt);
    } else {
        Stack st;
        st.lds = (CHR_LDS uint32_t *)(lds_stack + threadIdx.x);
        tri = intersect_mesh<4>(g, o, d, dist, -1, st, overflow);
    }
    if (tri != -1) distance[id] = dist;
    if (overflow && counters) atomicAdd(counters, overflow);
}

}  // namespace chr

// ====================================================================== C ABI
using namespace chr;

namespace {

inline unsigned grid_for(uint64_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

inline uint32_t scan_blocks(uint32_t nwords) { return (nwords + SCAN_WORDS - 1) / SCAN_WORDS; }

// word_offsets (nwords) + block prefixes (scan_blocks(nwords)) of the masks
void launch_mask_scan(const unsigned long long *masks, uint32_t nwords, uint32_t *word_offsets, uint32_t *block_sums,
                      uint32_t *out_counter, uint32_t *base, uint32_t *total_out, hipStream_t stream,
                      const uint32_t *dev_n = nullptr, const uint32_t *mode = nullptr, uint32_t skip = STEP_IDLE,
                      const HeadNext *hn = nullptr) {
    const uint32_t nb = scan_blocks(nwords);   // device-driven: nwords is an upper bound
    if (nb) hipLaunchKernelGGL(mask_block_scan_kernel, dim3(nb), dim3(SCAN_WORDS), 0, stream, masks, nwords, word_offsets,
                               block_sums, dev_n, mode, skip);
    hipLaunchKernelGGL(scan_block_sums_kernel, dim3(1), dim3(1024), 0, stream, block_sums, nb, out_counter, base,
                       total_out, mode, skip, dev_n ? 1u : 0u,
                       hn ? *hn : HeadNext{nullptr, nullptr, nullptr, nullptr, nullptr, 0u, 0u, 0, 0});
}

PhotonPtrs to_ptrs(const chr_photons *p) {
    return PhotonPtrs{p->d_pos, p->d_dir, p->d_pol, p->d_wavelengths, p->d_t, p->d_weights, p->d_flags,
                      p->d_last_hit_triangles, p->d_evidx};
}

bool photons_ok(const chr_photons *p) {
    return p && p->d_pos && p->d_dir && p->d_pol && p->d_wavelengths && p->d_t && p->d_weights && p->d_flags &&
           p->d_last_hit_triangles && p->d_evidx;
}

struct JumpTables {
    uint32_t *seq = nullptr, *off = nullptr;
    int device = -1;
};

int get_jump_tables(JumpTables &jt) {
    static thread_local JumpTables cache[16];
    int dev = 0;
    CHR_HIP_CHECK(hipGetDevice(&dev));
    if (dev < 0 || dev >= 16) return chr::fail(CHR_ERR_INVALID, "device id %d unsupported", dev);
    if (!cache[dev].seq) {
        static std::vector<uint32_t> hseq, hoff;
        if (hseq.empty()) {
            hseq.resize((size_t)CHR_XW_MATWORDS * 32);
            hoff.resize((size_t)CHR_XW_MATWORDS * 64);
            chr_xw_sequence_matrices(hseq.data(), 32);
            chr_xw_offset_matrices(hoff.data(), 64);
        }
        CHR_HIP_CHECK(hipMalloc(&cache[dev].seq, hseq.size() * 4));
        CHR_HIP_CHECK(hipMalloc(&cache[dev].off, hoff.size() * 4));
        CHR_HIP_CHECK(hipMemcpy(cache[dev].seq, hseq.data(), hseq.size() * 4, hipMemcpyHostToDevice));
        CHR_HIP_CHECK(hipMemcpy(cache[dev].off, hoff.data(), hoff.size() * 4, hipMemcpyHostToDevice));
    }
    jt = cache[dev];
    return CHR_OK;
}

// device scratch reused by the selection helpers (per thread, grown on demand)
struct Scratch {
    void *ptr = nullptr;
    size_t bytes = 0;
    int device = -1;
};

// ctx: which of a thread's NCTX propagate buffer contexts (chr_propagate_batches
// rotates them so batches can overlap: a tail, the next batches' first steps)
constexpr int NCTX = 3;
int scratch_get(size_t bytes, void **out, int ctx = 0) {
    static thread_local Scratch s[NCTX][16];
    int dev = 0;
    CHR_HIP_CHECK(hipGetDevice(&dev));
    Scratch &x = s[ctx % NCTX][dev & 15];
    if (x.bytes < bytes) {
        if (x.ptr) CHR_HIP_CHECK(hipFree(x.ptr));
        x.ptr = nullptr;
        CHR_HIP_CHECK(hipMalloc(&x.ptr, bytes));
        x.bytes = bytes;
    }
    *out = x.ptr;
    return CHR_OK;
}

// HBM column for the deep walk-stack entries of the persistent trace grid
// (per thread and device, grown on demand; see trace_kernel)
int walk_stack_get(size_t bytes, uint2 **out, int ctx = 0) {
    static thread_local Scratch s[NCTX][16];
    int dev = 0;
    CHR_HIP_CHECK(hipGetDevice(&dev));
    Scratch &x = s[ctx % NCTX][dev & 15];
    if (x.bytes < bytes) {
        if (x.ptr) CHR_HIP_CHECK(hipFree(x.ptr));
        x.ptr = nullptr;
        CHR_HIP_CHECK(hipMalloc(&x.ptr, bytes));
        x.bytes = bytes;
    }
    *out = (uint2 *)x.ptr;
    return CHR_OK;
}

}  // namespace

int chr::build_ref_triangles(const DevGeom &dg, float4 *tri) {
    if (!dg.wtri || !dg.nwtri) return chr::fail(CHR_ERR_INVALID, "build_ref_triangles: no wide triangle records");
    CHR_HIP_CHECK(hipMemset(tri, 0, (size_t)dg.ntriangles * 48));
    hipLaunchKernelGGL(ref_triangles_kernel, dim3(grid_for(dg.nwtri)), dim3(BLOCK), 0, 0, dg.wtri, dg.nwtri, tri);
    CHR_HIP_CHECK(hipGetLastError());
    CHR_HIP_CHECK(hipDeviceSynchronize());
    return CHR_OK;
}

extern "C" int chr_init_rng_subseq(uint32_t *d_states, uint32_t nslots, uint64_t seed, uint64_t first_subsequence,
                                   uint64_t offset, void *stream) {
    if (!d_states || nslots == 0) return chr::fail(CHR_ERR_INVALID, "chr_init_rng: empty state buffer");
    if (first_subsequence + nslots > (1ull << 32))
        return chr::fail(CHR_ERR_INVALID, "chr_init_rng: subsequences beyond 2^32 are not supported");
    JumpTables jt;
    int rc = get_jump_tables(jt);
    if (rc) return rc;
    hipLaunchKernelGGL(init_rng_kernel, dim3(grid_for(nslots)), dim3(BLOCK), 0, (hipStream_t)stream, d_states, nslots,
                       (unsigned long long)seed, (unsigned long long)first_subsequence, (unsigned long long)offset,
                       jt.seq, 32, jt.off, 64);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_init_rng(uint32_t *d_states, uint32_t nslots, uint64_t seed, uint64_t offset, void *stream) {
    return chr_init_rng_subseq(d_states, nslots, seed, 0, offset, stream);
}

extern "C" int chr_rng_download(const uint32_t *d_states, uint32_t nslots, uint32_t *h_out, void *stream) {
    CHR_HIP_CHECK(hipMemcpyAsync(h_out, d_states, (size_t)nslots * 24, hipMemcpyDeviceToHost, (hipStream_t)stream));
    CHR_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    return CHR_OK;
}

// the direction-binning sort's temporary storage (allocated for 24-bit keys, the largest
// CHR_BIN_KEY asks for; queried with the bits of the sort at hand)
static size_t sort_temp_bytes16(uint32_t n, int bits = 24) {
    size_t bytes = 0;
    (void)rocprim::radix_sort_pairs((void *)nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                    (const uint32_t *)nullptr, (uint32_t *)nullptr, n, 0, bits);
    return bytes;
}
// The first step's direction-binning sort: keys of 11+11-bit octahedral cells in
// Hilbert order (octa_cell).  r04 ab15/ab16/ab18 (29k bench, 10 M rays): the binned
// first launch 5.01 ms with r01-r03's 8+8-bit row-major cells, 4.63 with 11+11-bit
// Morton cells, 4.55 with Hilbert order (490.3 -> 500.3 M/s); photons identical.
constexpr int BIN_KEY_BITS = 22;
// u32 words: [0..15] counters | masks (2 per 64 slots) | offsets (1 per 64) |
// block prefixes (1 per 256 words, +2)
static uint64_t mask_scan_words(uint64_t n) {   // masks + offsets + block prefixes for n positions
    const uint64_t nwords = (n + 63) / 64;
    return 2 * nwords + nwords + scan_blocks((uint32_t)nwords) + 2;
}
extern "C" uint64_t chr_propagate_scratch_words(uint32_t nthreads) {
    return 16 + mask_scan_words(nthreads) + 64;
}

// Kernel variants (CHR_PROPAGATE_VARIANT=<n>, read per launch so one process
// can A/B them; every variant gives identical results -- tools/ab_variants.py
// checks histories, last hits and positions).  Measured choices: DESIGN.md
// section 5 and profiles/r01/ab_*.log.
//   0  default.  One-step launches: trace_kernel (BVH walk, first step's rays
//      binned by direction) + shade_kernel<3>; multi-step launches (the tail):
//      propagate_tail_kernel (wave-adaptive walk, 8 lanes of physics per photon).
//   5  counting form of 0 (bench: node/triangle counts of the walk); its
//      multi-step launches run the counting fused kernel.
//   1  exact-order walk of the reference BVH (fused step kernel).
//   2  fused step kernel with the speculative wide walk (walk + physics per
//      lane: the design the split replaced); 3 = its counting form.
//   4  scheduled wide walk (fused); used automatically when the triangle
//      records do not fit the 30-bit leaf queue; 6 = its counting form.
//   7  the split with binning on every step; 8 the split without binning.
typedef void (*propagate_fn)(const DevGeom *, PropagateArgs);
static constexpr int kWalk = 2006;        // speculative wide walk, triangle steps at 6/8 of the live lanes
static constexpr int kWalkSched = 1002;   // scheduled wide walk, triangle batch 2
static constexpr int kExactVariant = 1;
// propagate_tail_kernel (wave-adaptive walk) at 2 waves/SIMD: ~200 VGPRs, no
// spills, no private segment.  r03 A/B on the 29k bench (profiles/r03/ab3, same
// batches and RNG for every configuration): the long-lived photon's step 26.7 ->
// 21.5 us, mean tail 7.31 -> 6.64 ms against 3 waves/SIMD (168 VGPRs, 51 spilled
// once the GS = 64 walk was added); r02 measured 3 waves ahead of 4 (64 spills).
static constexpr int kTailWaves = 2;
// The shade and tail kernels copy the physics tables into LDS (phys_cache): r03
// ab16, 29k bench, 450.7 -> 461.7 M/s, mean tail 6.36 -> 6.06 ms.  The tail kernel's
// walks read the top of the tree from LDS (stage_top): walk 16.4 -> 16.0 us per step
// of the long-lived photon (r04 ab1).  The shade kernel reads queue entries two ahead
// and never waits for its own write-back (shade_kernel, r04 ab9/ab10).  A wave of the
// tail kernel with one walking photon walks it with walk_lone (r04 §10.1: 474.6 ->
// 489.4 M/s against walk_segment<64>), as does a trace wave draining one walk.
// trace_kernel waves drain their last <= 4 walks whole-wave (r03 ab3: trace ms per
// step 16.23 at 8, 15.92 at 2, 15.90 at 4, 16.33 off): each then has >= 2 cursors.
static bool wide_queue_ok(const chr_geometry *g) { return g->dev.nwtri < (1u << 30); }   // 30-bit leaf queue entries

// whether this call's kernels walk the reference BVH (its nodes must be resident)
static bool walks_reference_bvh(const chr_geometry *g) {
    const char *e = getenv("CHR_PROPAGATE_VARIANT");
    return g->dev.nwnodes == 0 || (e && atoi(e) == kExactVariant);
}

static propagate_fn select_variant(const chr_geometry *g) {
    const char *e = getenv("CHR_PROPAGATE_VARIANT");
    int v = e ? atoi(e) : 0;
    if (g->dev.nwnodes == 0) v = kExactVariant;   // no wide BVH for this geometry
    const bool counting = (v == 3 || v == 5 || v == 6);
    if (v == kExactVariant) return propagate_kernel<8, 4, 0>;
    if (v == 4 || v == 6 || !wide_queue_ok(g))
        return counting ? propagate_kernel<8, 4, kWalkSched, true> : propagate_kernel<8, 4, kWalkSched>;
    return counting ? propagate_kernel<8, 4, kWalk, true> : propagate_kernel<8, 4, kWalk>;
}

typedef void (*propagate_step_fn)(const DevGeom *, PropagateArgs, uint32_t);
typedef void (*trace_fn)(const DevGeom *, TraceArgs);
struct StepVariant {
    propagate_step_fn fn;           // fused step kernel (any max_steps)
    trace_fn trace = nullptr;       // one-step launches: trace_kernel + shade (nullptr: fn)
    trace_fn trace_gather = nullptr;   // its form refilling from the photon arrays (no ray records)
    propagate_step_fn shade = nullptr;
    int trace_waves = 4;            // waves per SIMD of the trace kernel (persistent grid size)
    int trace_block = BLOCK;        // its workgroup size
    propagate_step_fn tail = nullptr;   // multi-step launches: group-walk kernel (nullptr: fn)
    int tail_group = 0;                 // its lanes per photon
    int binned = 0;                 // trace order binned by direction: 1 every step, 2 first host step only
};
// Direction binning pays where the rays of a step share an origin -- the
// first step of a point or track source -- and not after the first bounce
// (demo.detector(), 4M photons: first-step walk 2.65 -> 2.21 ms for 0.11 ms of
// sorting; second step unchanged).
static constexpr uint32_t kBinFirstMin = 1u << 20;
// Measured and removed (records in DESIGN 9-10): claim-ahead ray-counter chunks (r03
// ab5, r04 ab14: slower, the counter is not contended), a 1024-thread trace layout with
// the top of the tree in LDS (r04 ab1: no gain), refill thresholds other than 48 (r03
// ab3: 17.87 at 16, 16.25 at 32, 15.81 ms per step at 48; r04 ab12: 14.45 at 56, 17.36
// at 64), prefetched rays per lane (r04 ab11: every launch 30-40% longer), five node
// loads instead of six (r04 ab7), 5 waves per SIMD (r04 ab6), a combined node + triangle
// step (r04 ab3), the walk-order carry (r03 ab10/ab14, r04 ab17: the walk-order scatter
// cost more than the walks gained), a coherence sort of every launch (r01).
static StepVariant select_step_variant(const chr_geometry *g) {
    const char *e = getenv("CHR_PROPAGATE_VARIANT");
    int v = e ? atoi(e) : 0;
    const bool wires = g->dev.nwireplanes > 0;   // shade / tail without the wire-plane code otherwise
    StepVariant sv;
    if (g->dev.nwnodes == 0 || v == kExactVariant) {
        sv.fn = propagate_step_kernel<8, 4, 0>;
        return sv;
    }
    if (!wide_queue_ok(g) || v == 4 || v == 6) {
        sv.fn = (v == 3 || v == 5 || v == 6) ? propagate_step_kernel<8, 4, kWalkSched, true>
                                              : propagate_step_kernel<8, 4, kWalkSched>;
        return sv;
    }
    switch (v) {
        case 2: sv.fn = propagate_step_kernel<8, 4, kWalk>; break;
        case 3: sv.fn = propagate_step_kernel<8, 4, kWalk, true>; break;
        case 5:   // walk counters of the one-step launches' trace kernel; the tail as variant 0
            sv.fn = propagate_step_kernel<8, 4, kWalk, true>;
            sv.trace = trace_kernel<true, 6, 12, 4, 32>;
            sv.trace_gather = trace_kernel<true, 6, 12, 4, 32, true>;
            sv.shade = wires ? shade_kernel<3> : shade_kernel<3, false>;
            sv.tail = wires ? propagate_tail_kernel<kTailWaves> : propagate_tail_kernel<kTailWaves, false>;
            sv.tail_group = 8;
            sv.binned = 2;
            break;
        default:   // 0, 7, 8
            sv.fn = propagate_step_kernel<8, 4, kWalk>;
            sv.trace = trace_kernel<false, 6, 12, 4, 48>;
            sv.trace_gather = trace_kernel<false, 6, 12, 4, 48, true>;
            sv.shade = wires ? shade_kernel<3> : shade_kernel<3, false>;
            sv.tail = wires ? propagate_tail_kernel<kTailWaves> : propagate_tail_kernel<kTailWaves, false>;
            sv.tail_group = 8;
            sv.binned = v == 7 ? 1 : (v == 8 ? 0 : 2);
            break;
    }
    // the physics tables' LDS copy is dynamic LDS (phys_lds_bytes): allow the caps, once
    static const bool lds_caps = []() {
        const int sb = (int)(SHADE_PHYS_WORDS * 4), tb = (int)(TAIL_PHYS_WORDS * 4);
        (void)hipFuncSetAttribute((const void *)shade_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, sb);
        (void)hipFuncSetAttribute((const void *)shade_kernel<3, false>, hipFuncAttributeMaxDynamicSharedMemorySize, sb);
        (void)hipFuncSetAttribute((const void *)propagate_tail_kernel<kTailWaves>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, tb);
        (void)hipFuncSetAttribute((const void *)propagate_tail_kernel<kTailWaves, false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, tb);
        (void)hipGetLastError();
        return true;
    }();
    (void)lds_caps;
    return sv;
}

// scratch layout (u32 words): [0] overflows [1] queue base [2..11] u64 walk counters [12..15] pad; masks (u64, 8-aligned); offsets
static bool pair_walk_enabled();
static uint32_t walk_up_mode();
static int launch_chunk(const chr_geometry *g, const chr_photons *ph, uint32_t *rng, uint32_t nslots, int32_t first,
                        int32_t nthreads, const uint32_t *in_queue, uint32_t *out_queue, int32_t max_steps,
                        int32_t use_weights, int32_t scatter_first, uint32_t *scratch, hipStream_t stream,
                        hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr) {
    const uint32_t nwords = (uint32_t)((nthreads + 63) / 64);
    uint32_t *counters = scratch;               // [0] overflows, [1] base
    unsigned long long *masks = (unsigned long long *)(scratch + 16);
    uint32_t *offsets = scratch + 16 + 2 * (size_t)nwords;
    uint32_t *bsums = offsets + nwords;
    PropagateArgs a;
    a.pos = ph->d_pos; a.dir = ph->d_dir; a.pol = ph->d_pol; a.wl = ph->d_wavelengths; a.t = ph->d_t;
    a.weights = ph->d_weights; a.flags = ph->d_flags; a.last_hit = ph->d_last_hit_triangles; a.evidx = ph->d_evidx;
    a.rng = rng; a.nslots = nslots; a.input_queue = in_queue; a.first = first; a.nthreads = nthreads;
    a.max_steps = max_steps; a.use_weights = use_weights; a.scatter_first = scatter_first;
    a.alive_masks = masks; a.counters = counters;
    a.order = nullptr;
    a.hits = nullptr;
    a.diag = nullptr;
    a.dev_n = nullptr;
    a.mode = nullptr;
    a.want = STEP_ONE;
    a.work = nullptr;
    a.prio = 0;
    a.pair = pair_walk_enabled() ? 1u : 0u;
    a.walk_up = walk_up_mode();
    if (ev0) CHR_HIP_CHECK(hipEventRecord(ev0, stream));
    hipLaunchKernelGGL(select_variant(g), dim3(grid_for(nthreads)), dim3(BLOCK), 0, stream,
                       (const DevGeom *)g->d_dev, a);
    if (ev1) CHR_HIP_CHECK(hipEventRecord(ev1, stream));
    launch_mask_scan(masks, nwords, offsets, bsums, out_queue, counters + 1, nullptr, stream);
    hipLaunchKernelGGL(scatter_queue_kernel, dim3(grid_for(nthreads)), dim3(BLOCK), 0, stream, masks, offsets, bsums,
                       counters + 1, in_queue, first, nthreads, out_queue,
                       RayEnrol{nullptr, nullptr, nullptr, nullptr}, (const uint32_t *)nullptr,
                       (const uint32_t *)nullptr, STEP_IDLE);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

// one host step as one launch of propagate_step_kernel over the n queued
// photons (slot = queue position mod cap); same scratch layout as launch_chunk
// with mask words per queue position.
static int device_cus() {
    static int cus[16] = {};
    int dev = 0;
    CHR_HIP_CHECK(hipGetDevice(&dev));
    if (!cus[dev & 15]) CHR_HIP_CHECK(hipDeviceGetAttribute(&cus[dev & 15], hipDeviceAttributeMultiprocessorCount, dev));
    return cus[dev & 15];
}

// Split-step bookkeeping of one propagate (trace_kernel): control words --
// ctl[3] flat rays walked by the trace kernel, ctl[4] flat rays walked by the
// multi-step kernels (diagnostics; rounds 2-4 decomposed flat walks into
// sub-walks, §11.6) -- and the ray records.
struct FlatCtx {
    uint32_t *ctl;
    bool enrol_next;
    // trace_kernel's ray records (put_ray): rays in queue order (the first
    // step's classification, then every step's scatter for the next step),
    // rays_walk the binned first step's records permuted into walk order
    uint4 *rays = nullptr, *rays_walk = nullptr;
};
static int flat_get(uint32_t n, FlatCtx &fc, int ctx = 0) {
    static thread_local Scratch s[NCTX][16];
    int dev = 0;
    CHR_HIP_CHECK(hipGetDevice(&dev));
    Scratch &x = s[ctx % NCTX][dev & 15];
    (void)n;
    const size_t bytes = 256;
    if (x.bytes < bytes) {
        if (x.ptr) CHR_HIP_CHECK(hipFree(x.ptr));
        x.ptr = nullptr;
        CHR_HIP_CHECK(hipMalloc(&x.ptr, bytes));
        x.bytes = bytes;
    }
    fc.ctl = (uint32_t *)x.ptr;
    fc.enrol_next = false;
    return CHR_OK;
}

static bool trace_steps();
// CHR_SLOT_TIMING: which per-slot timing events a device-driven propagate
// records.  Each hipEventRecord between two dependent dispatches of a step's
// chain adds a gap (r03 ab15, 29k bench: all 449.9, trace pair only 452.6,
// none 454.7 M/s).  Default "trace": only the pair around each trace launch
// (the stats' trace_ms / trace_launch_ms, which the bench's roofline uses);
// "1" every slot's events as well (kernel_ms, tail_ms, the prefix split);
// "0" only the events the streams and the host synchronise on.  Times not
// recorded read 0 in chr_propagate_stats.
// CHR_PAIR_WALK=0: the tail's lone walks on their own wave only (walk_lone; A/B,
// default 1: walk_pair with an idle wave of the workgroup as tester)
static bool pair_walk_enabled() {
    const char *e = getenv("CHR_PAIR_WALK");
    return !(e && e[0] == '0');
}
// CHR_WALK_UP=0: the tail's walks from the root (A/B; default 1: a walk with a
// previous hit climbs from that hit's leaf -- walk_lone<true> ahead of the pair walk,
// and the grouped walks, walk_segment<0, UP>, the lone walk's first iteration taking the
// start node's ancestors read during the previous step; 2: the lone walks only; 4: as 1
// without that prefetch -- A/B)
static uint32_t walk_up_mode() {
    const char *e = getenv("CHR_WALK_UP");
    return e && (e[0] == '0' || e[0] == '2' || e[0] == '4') ? (uint32_t)(e[0] - '0') : 1u;
}

static int slot_timing() {
    const char *e = getenv("CHR_SLOT_TIMING");
    if (!e || e[0] == 't') return 1;
    if (e[0] == '0') return 0;
    return 2;
}
// A device-driven step slot (chr_propagate without a host round trip per
// step): the slot's kernels read the queue length from the input queue's
// header and run by the mode step_head_kernel picks; n passed to launch_step
// is then an upper bound that sizes grids and scratch.
struct SlotCtl {
    uint32_t *mode;        // this slot's mode word (device)
    uint32_t *nk;          // this slot's queue length, written by the head kernel (device)
    uint32_t *done;        // set once the queue is empty or the tail ran (device)
    uint32_t n_layout;     // photons of the propagate: layout of the hits / binning regions
    int32_t remaining;     // steps left (max_steps - step)
    uint32_t tail_below;   // the nsteps policy's threshold, nthreads_per_block * 128
    // chr_propagate_batches: the slot's tail kernel runs on its own stream
    // (after the slot's trace-start event, or its one-step kernels' ev1 with every
    // slot event recorded), so the caller's stream moves on
    // to the next batch while a tail's long-lived photons finish.  The tail
    // leaves no queue (it runs every remaining step): its alive bits go to
    // tail_masks and the slot's scan / scatter skip the tail mode.
    hipStream_t tail_stream = nullptr;
    unsigned long long *tail_masks = nullptr;
    hipEvent_t evt_tail0 = nullptr, evt_tail1 = nullptr;   // around the tail kernel, on tail_stream
    hipEvent_t rng_ready = nullptr;   // the previous batch's tail done: the first RNG use waits for it
    // chr_propagate_batches runs a batch's first slot in two parts: PHASE_PREFIX
    // (head, flat-walk classification, binning, the BVH walk: no random numbers)
    // on the prefix stream, ending with prefix_done; PHASE_REST (shade pass on)
    // on the batch stream after prefix_done, starting with ev_rest0
    int phase = 0;
    int ctx = 0;                      // buffer context (walk-stack column)
    uint32_t *host_ring = nullptr;    // pinned (mode, length) words the head kernel writes (nullptr: none)
    // the next slot's head folded into this slot's block-sum scan (fold_head: every slot
    // after the first then launches no head kernel of its own); next_head.ray_counter is
    // filled by launch_step
    bool fold_head = false;
    HeadNext next_head{nullptr, nullptr, nullptr, nullptr, nullptr, 0u, 0u, 0, 0};
    hipEvent_t prefix_done = nullptr, ev_rest0 = nullptr;
};
constexpr int PHASE_ALL = 0, PHASE_PREFIX = 1, PHASE_REST = 2;

// The wave-adaptive tail kernel as one resident grid whose photon groups take
// queue positions from a counter (PropagateArgs::work; the slot's ray counter,
// zeroed by the head kernel) -- where every queued photon has its own RNG slot
// (the tail starts below nthreads_per_block * 128 photons and that is at most
// the slot count; not use_weights, whose tail takes any length).  r03 ab11, 29k
// bench: 440.4 -> 450.3 M/s (mean tail 6.93 -> 6.65 ms, kernel time per step
// 29.98 -> 28.37 ms).  CHR_TAIL_WQ=0: one group per slot, as many waves as
// photons / 8.
static bool tail_work_queue(const StepVariant &sv, const SlotCtl *sc, int32_t use_weights, uint32_t cap) {
    return sv.tail_group == 8 && sc && !use_weights && sc->tail_below <= cap;
}
// blocks of a tail launch: every slot's group, or (work queue) the resident grid
static unsigned tail_grid(const StepVariant &sv, uint32_t threads, bool work_queue) {
    const unsigned full = grid_for((uint64_t)threads * sv.tail_group);
    if (!work_queue) return full;
    const int cus = device_cus();
    const unsigned resident = (unsigned)std::max(1, cus) * (unsigned)kTailWaves * 4u * 64u / BLOCK;
    return std::max(1u, std::min(full, resident));
}

static int launch_step(const chr_geometry *g, const chr_photons *ph, uint32_t *rng, uint32_t nslots, uint32_t cap,
                       uint32_t n, const uint32_t *in_queue, uint32_t *out_queue, int32_t max_steps,
                       int32_t use_weights, int32_t scatter_first, uint32_t *scratch, hipStream_t stream,
                       hipEvent_t ev0, hipEvent_t ev1, int2 *hits, uint32_t *sort_space, bool first_step,
                       hipEvent_t evt0, hipEvent_t evt1, bool *split_out, const FlatCtx *fc,
                       const SlotCtl *sc = nullptr) {
    const uint32_t nwords = (n + 63) / 64;
    uint32_t *counters = scratch;
    unsigned long long *masks = (unsigned long long *)(scratch + 16);
    uint32_t *offsets = scratch + 16 + 2 * (size_t)nwords;
    uint32_t *bsums = offsets + nwords;
    const uint32_t *dev_n = sc ? in_queue - 1 : nullptr;   // the input queue's count header
    const uint32_t *mode = sc ? sc->mode : nullptr;
    PropagateArgs a;
    a.pos = ph->d_pos; a.dir = ph->d_dir; a.pol = ph->d_pol; a.wl = ph->d_wavelengths; a.t = ph->d_t;
    a.weights = ph->d_weights; a.flags = ph->d_flags; a.last_hit = ph->d_last_hit_triangles; a.evidx = ph->d_evidx;
    a.rng = rng; a.nslots = nslots; a.input_queue = in_queue; a.first = 0; a.nthreads = (int32_t)n;
    a.max_steps = max_steps; a.use_weights = use_weights; a.scatter_first = scatter_first;
    a.alive_masks = masks; a.counters = counters;
    a.order = nullptr;
    a.hits = nullptr;
    a.diag = fc ? fc->ctl + 4 : nullptr;
    a.dev_n = dev_n;
    a.mode = mode;
    a.want = STEP_ONE;
    a.work = nullptr;
    a.prio = 0;
    a.pair = pair_walk_enabled() ? 1u : 0u;
    a.walk_up = walk_up_mode();
    RayEnrol fe{nullptr, nullptr, nullptr, nullptr};
    const uint32_t threads = std::min(cap, (n + 63u) & ~63u);
    const StepVariant sv = select_step_variant(g);
    // host-driven: the split when this launch is one step; device-driven: the
    // one-step kernels and the tail kernel are both queued and the head picks
    const bool split = sv.trace && hits && fc && (sc ? true : max_steps == 1);
    const bool tail = sv.tail && (sc ? sc->remaining > 1 : (!split && max_steps > 1));
    // the first step's length and mode are known on the host (binning, flat-walk enrolment)
    const bool first_one_step = first_step && (!sc || !((n < sc->tail_below || use_weights) && sc->remaining > 1));
    uint32_t *next = split ? (uint32_t *)(hits + (sc ? sc->n_layout : n)) : nullptr;
    const int phase = sc ? sc->phase : PHASE_ALL;
    const bool pre = phase != PHASE_REST, rest = phase == PHASE_ALL || phase == PHASE_REST;
    if (phase != PHASE_ALL && (!split || !sc->prefix_done))
        return chr::fail(CHR_ERR_INVALID, "launch_step: a split slot needs the split path and its prefix event");
    if (ev0 && pre) CHR_HIP_CHECK(hipEventRecord(ev0, stream));
    if (!pre) {
        CHR_HIP_CHECK(hipStreamWaitEvent(stream, sc->prefix_done, 0));
        if (sc->ev_rest0) CHR_HIP_CHECK(hipEventRecord(sc->ev_rest0, stream));
    }
    // the next slot's head, folded into this slot's scan (SlotCtl::fold_head)
    HeadNext hn{nullptr, nullptr, nullptr, nullptr, nullptr, 0u, 0u, 0, 0};
    if (sc && sc->fold_head && sc->next_head.mode && next) {
        hn = sc->next_head;
        hn.ray_counter = next;
    }
    const HeadNext *hnp = hn.mode ? &hn : nullptr;
    if (sc && pre && !(sc->fold_head && !first_step)) {
        if (!next) return chr::fail(CHR_ERR_INVALID, "launch_step: device-driven steps need the split path");
        hipLaunchKernelGGL(step_head_kernel, dim3(1), dim3(64), 0, stream, in_queue - 1, out_queue, sc->mode, sc->nk,
                           sc->done, next, sc->tail_below, sc->remaining, use_weights, sc->n_layout, sc->host_ring);
    } else if (split && !sc) {
        CHR_HIP_CHECK(hipMemsetAsync(next, 0, 4, stream));
    }
    if (split) {
        // direction binning: 16-bit radix sort of (direction cell, queue position); hits region:
        // [hits n x int2][next + pad, 16 words][keys n][values n][walk hist 64 words]
        // (device-driven slots bin only the first step, whose length the host knows)
        const bool binned = (sv.binned == 1 || (sv.binned == 2 && first_one_step && n >= kBinFirstMin)) &&
                            (!sc || first_one_step);
        const bool bin_now = binned && pre;
        uint32_t *keys = next + 16, *order = keys + n;
        // ray records: the first step's from its classification, later steps' from
        // the previous step's scatter (enrol_next)
        const bool use_rays = fc->rays && (first_one_step || fc->enrol_next);
        if (first_one_step && pre)   // the initial queue's ray records and keys (later steps: the previous scatter)
            hipLaunchKernelGGL(classify_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, stream, ph->d_pos, ph->d_dir,
                               ph->d_flags, ph->d_last_hit_triangles, in_queue, n, bin_now ? keys : nullptr,
                               bin_now ? order : nullptr, use_rays ? fc->rays : nullptr);
        TraceArgs ta;
        ta.pos = ph->d_pos; ta.dir = ph->d_dir; ta.flags = ph->d_flags; ta.last_hit = ph->d_last_hit_triangles;
        ta.queue = in_queue; ta.n = n; ta.hits = hits; ta.next = next; ta.counters = counters; ta.order = nullptr;
        ta.rays = use_rays ? fc->rays : nullptr;
        ta.walk_hist = nullptr;
        ta.diag = fc->ctl + 3;
        ta.dev_n = dev_n;
        ta.mode = mode;
        if (fc->enrol_next) fe = RayEnrol{ph->d_pos, ph->d_dir, fc->rays, ph->d_last_hit_triangles};
        if (trace_steps() && pre) {   // debugging: per-walk cost histogram (counting variants), printed per step
            ta.walk_hist = next + 16 + 2 * (size_t)(sc ? sc->n_layout : n);
            CHR_HIP_CHECK(hipMemsetAsync(ta.walk_hist, 0, 34 * 4, stream));
        }
        if (binned) {
            uint32_t *keys_out = sort_space, *vals_out = keys_out + n;
            if (bin_now) {
                if (!first_one_step)   // the first step's keys came with its classification
                    hipLaunchKernelGGL(bin_key_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, stream, ph->d_dir, in_queue,
                                       n, keys, order);
                void *temp = (void *)(((uintptr_t)(vals_out + n) + 255) & ~(uintptr_t)255);
                size_t temp_bytes = sort_temp_bytes16(n, BIN_KEY_BITS);
                CHR_HIP_CHECK(rocprim::radix_sort_pairs(temp, temp_bytes, keys, keys_out, order, vals_out, n, 0,
                                                        BIN_KEY_BITS, stream));
                if (use_rays)   // the records in the binned walk order
                    hipLaunchKernelGGL(permute_rays_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, stream, fc->rays,
                                       vals_out, n, fc->rays_walk);
            }
            ta.order = vals_out;
            if (use_rays) ta.rays = fc->rays_walk;
        }
        if (pre) {
            const int cus = device_cus();
            if (cus <= 0) return chr::fail(CHR_ERR_HIP, "launch_step: no compute units");
            const int tb = sv.trace_block;
            const uint64_t resident = (uint64_t)cus * 4 * sv.trace_waves * 64 / tb;   // persistent grid
            const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(resident, ((uint64_t)n + tb - 1) / tb));
            if (int rc = walk_stack_get((size_t)WIDE_STACK * blocks * tb * sizeof(uint2), &ta.spill, sc ? sc->ctx : 0))
                return rc;
            if (evt0) CHR_HIP_CHECK(hipEventRecord(evt0, stream));
            hipLaunchKernelGGL(ta.rays ? sv.trace : sv.trace_gather, dim3(blocks), dim3(tb), 0, stream,
                               (const DevGeom *)g->d_dev, ta);
            if (evt1) CHR_HIP_CHECK(hipEventRecord(evt1, stream));
        }
        if (!rest) {
            CHR_HIP_CHECK(hipEventRecord(sc->prefix_done, stream));
            CHR_HIP_CHECK(hipGetLastError());
            return CHR_OK;
        }
        a.hits = hits;
        a.max_steps = 1;
        if (sc && sc->rng_ready) CHR_HIP_CHECK(hipStreamWaitEvent(stream, sc->rng_ready, 0));
        hipLaunchKernelGGL(sv.shade, dim3(grid_for(threads)), dim3(BLOCK), phys_lds_bytes(g->dev, SHADE_PHYS_WORDS), stream,
                           (const DevGeom *)g->d_dev, a, cap);
    }
    if (split_out) *split_out = split;
    if (tail && sc && sc->tail_stream) {   // the tail on its own stream (chr_propagate_batches)
        // the tail kernel needs the slot's head (its mode) and the previous slot's scatter (its
        // queue): both come before the slot's trace-start event; with every slot event
        // recorded (CHR_SLOT_TIMING=1) it waits for the slot's one-step part as before.
        // Invariant that makes the earlier event enough: every kernel queued on `stream`
        // for this slot (classify / binning, trace, shade, scan, scatter) exits at once
        // when the slot's mode is STEP_TAIL (their mode / want checks), so none of them
        // touches the photons, queues or RNG slots the tail works on; and the RNG slot
        // states the tail reads were last written by kernels ordered before ev0 on
        // `stream`, or by the previous batch's tail, earlier on this same tail stream.
        // tests/test_gpu_batches.py checks CHR_SLOT_TIMING=0 / 1 give identical photons.
        hipEvent_t dep = ev1 ? ev1 : evt0;
        if (!dep) return chr::fail(CHR_ERR_INVALID, "launch_step: a tail stream needs a slot event");
        hipStream_t ts = sc->tail_stream;
        if (ev1) CHR_HIP_CHECK(hipEventRecord(ev1, stream));
        CHR_HIP_CHECK(hipStreamWaitEvent(ts, dep, 0));
        if (sc->evt_tail0) CHR_HIP_CHECK(hipEventRecord(sc->evt_tail0, ts));
        // few workgroups (grid-stride): a tail holds < nthreads_per_block * 128 photons
        // unless use_weights, and this launch waits for free CU slots beside the
        // next batch's persistent walk grid -- a 1024-workgroup clear measured
        // 125 us per slot (r03 rocprof), every slot's on the tail's stream
        hipLaunchKernelGGL(clear_masks_kernel, dim3(std::min<uint32_t>(kClearBlocks, grid_for(nwords))), dim3(BLOCK), 0, ts,
                           sc->tail_masks, dev_n, mode);
        PropagateArgs at = a;
        at.prio = 1u;
        at.alive_masks = sc->tail_masks;
        at.max_steps = sc->remaining;
        at.want = STEP_TAIL;
        at.work = tail_work_queue(sv, sc, use_weights, cap) ? next : nullptr;
        hipLaunchKernelGGL(sv.tail, dim3(tail_grid(sv, threads, at.work != nullptr)), dim3(BLOCK),
                           phys_lds_bytes(g->dev, TAIL_PHYS_WORDS), ts,
                           (const DevGeom *)g->d_dev, at, cap);
        if (sc->evt_tail1) CHR_HIP_CHECK(hipEventRecord(sc->evt_tail1, ts));
        launch_mask_scan(masks, nwords, offsets, bsums, out_queue, counters + 1, nullptr, stream, dev_n, mode, STEP_TAIL,
                         hnp);
        hipLaunchKernelGGL(scatter_queue_kernel, dim3(std::min<uint32_t>(4096u, grid_for(n))), dim3(BLOCK), 0, stream,
                           masks, offsets, bsums, counters + 1, in_queue, 0, (int32_t)n, out_queue, fe, dev_n, mode,
                           STEP_TAIL);
        CHR_HIP_CHECK(hipGetLastError());
        return CHR_OK;
    }
    if (tail) {   // group / wave-adaptive walk, alive bits OR-ed into zeroed words
        if (sc) hipLaunchKernelGGL(clear_masks_kernel, dim3(std::min<uint32_t>(kClearBlocks, grid_for(nwords))), dim3(BLOCK), 0,
                                   stream, masks, dev_n, mode);
        else CHR_HIP_CHECK(hipMemsetAsync(masks, 0, (size_t)nwords * 8, stream));
        a.max_steps = sc ? sc->remaining : max_steps;
        a.want = STEP_TAIL;
        a.work = (sc && next && tail_work_queue(sv, sc, use_weights, cap)) ? next : nullptr;
        hipLaunchKernelGGL(sv.tail, dim3(tail_grid(sv, threads, a.work != nullptr)), dim3(BLOCK),
                           phys_lds_bytes(g->dev, TAIL_PHYS_WORDS), stream,
                           (const DevGeom *)g->d_dev, a, cap);
    } else if (!split) {
        hipLaunchKernelGGL(sv.fn, dim3(grid_for(threads)), dim3(BLOCK), 0, stream, (const DevGeom *)g->d_dev, a, cap);
    }
    if (ev1) CHR_HIP_CHECK(hipEventRecord(ev1, stream));
    launch_mask_scan(masks, nwords, offsets, bsums, out_queue, counters + 1, nullptr, stream, dev_n, mode, STEP_IDLE, hnp);
    hipLaunchKernelGGL(scatter_queue_kernel, dim3(sc ? std::min<uint32_t>(4096u, grid_for(n)) : grid_for(n)), dim3(BLOCK),
                       0, stream, masks, offsets, bsums, counters + 1, in_queue, 0, (int32_t)n, out_queue, fe, dev_n,
                       mode, STEP_IDLE);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_propagate_chunk(const chr_geometry *g, const chr_photons *ph, uint32_t *d_rng_states,
                                   uint32_t rng_nslots, int32_t first_photon, int32_t nthreads,
                                   const uint32_t *d_input_queue, uint32_t *d_output_queue, int32_t max_steps,
                                   int32_t use_weights, int32_t scatter_first, uint32_t *d_scratch, void *stream) {
    if (!g || !photons_ok(ph) || !d_rng_states || !d_input_queue || !d_output_queue || !d_scratch)
        return chr::fail(CHR_ERR_INVALID, "chr_propagate_chunk: null argument");
    if (nthreads <= 0) return CHR_OK;
    if ((uint32_t)nthreads > rng_nslots)
        return chr::fail(CHR_ERR_INVALID, "chr_propagate_chunk: %d threads but only %u rng states", nthreads, rng_nslots);
    if (walks_reference_bvh(g)) CHR_TRY(chr::geometry_ref_nodes(g));
    return launch_chunk(g, ph, d_rng_states, rng_nslots, first_photon, nthreads, d_input_queue, d_output_queue,
                        max_steps, use_weights, scatter_first, d_scratch, (hipStream_t)stream);
}

// pinned host words for survivor counts / counters (per thread and device, reused)
static int pinned_words(uint32_t **out, int ctx = 0) {
    static thread_local uint32_t *p[2][16] = {};
    int dev = 0;
    CHR_HIP_CHECK(hipGetDevice(&dev));
    uint32_t *&w = p[ctx & 1][dev & 15];
    if (!w) CHR_HIP_CHECK(hipHostMalloc((void **)&w, 512, hipHostMallocDefault));
    *out = w;
    return CHR_OK;
}

// timing events, reused across calls (per thread)
static int timing_events(size_t n, std::vector<hipEvent_t> **out, int ctx = 0) {
    static thread_local std::vector<hipEvent_t> ev[2][16];
    int dev = 0;
    CHR_HIP_CHECK(hipGetDevice(&dev));
    std::vector<hipEvent_t> &v = ev[ctx & 1][dev & 15];
    while (v.size() < n) {
        hipEvent_t e;
        CHR_HIP_CHECK(hipEventCreate(&e));
        v.push_back(e);
    }
    *out = &v;
    return CHR_OK;
}

static bool trace_steps() {   // CHR_TRACE_STEPS=1: one stderr line per host step (debugging)
    const char *e = getenv("CHR_TRACE_STEPS");
    return e && e[0] == '1';
}

static bool step_launch_enabled() {   // CHR_STEP_LAUNCH=0: the reference's one-launch-per-chunk structure (A/B)
    const char *e = getenv("CHR_STEP_LAUNCH");
    return !(e && e[0] == '0');
}

static bool host_steps_forced() {     // CHR_HOST_STEPS=1: read the survivor count on the host every step (A/B)
    const char *e = getenv("CHR_HOST_STEPS");
    return e && e[0] == '1';
}

// per-slot control words of a device-driven propagate: [2k] mode, [2k + 1]
// queue length of slot k, then the done flag (per thread and device, grown on demand)
static int slot_ctl_get(size_t words, uint32_t **out, int ctx = 0) {
    static thread_local Scratch s[NCTX][16];
    int dev = 0;
    CHR_HIP_CHECK(hipGetDevice(&dev));
    Scratch &x = s[ctx % NCTX][dev & 15];
    if (x.bytes < words * 4) {
        if (x.ptr) CHR_HIP_CHECK(hipFree(x.ptr));
        x.ptr = nullptr;
        CHR_HIP_CHECK(hipMalloc(&x.ptr, words * 4));
        x.bytes = words * 4;
    }
    *out = (uint32_t *)x.ptr;
    return CHR_OK;
}

// per-slot events of a device-driven propagate: [0] slot start, [1] its
// one-step kernels done (with the tail when that runs on the same stream),
// [2,3] around trace_kernel, [4] slot done (ring copied), [5,6] around the tail
// kernel when it runs on the tail stream, [7] start of the rest of a slot whose
// prefix ran on the prefix stream (chr_propagate_batches)
constexpr int SLOT_EVENTS = 8;

// Device buffers of one propagate (context ctx of the calling thread):
// queues, step scratch, the split path's hits / binning region, the flat-walk
// lists, and (tail_masks) alive words for a tail run on its own stream.
struct PropBufs {
    uint64_t cap = 0;        // slots of one chunk, nthreads_per_block * max_blocks
    bool fused = false;      // one launch per step
    uint32_t *q[2] = {nullptr, nullptr};
    uint32_t *scratch = nullptr;
    int2 *hits = nullptr;
    uint32_t *sort_space = nullptr;
    unsigned long long *tail_masks = nullptr;
    uint32_t *pinned = nullptr;
    FlatCtx fc{};
};

static int prop_bufs(uint32_t nphotons, int32_t ntpb, int32_t max_blocks, int ctx, bool tail_masks, PropBufs &b) {
    b.cap = (uint64_t)ntpb * max_blocks;   // slots of one chunk (chunk_iterator)
    const uint32_t chunk_cap = (uint32_t)std::min<uint64_t>(b.cap, nphotons);
    // one launch per step when a wave's 64 slots map to whole mask words
    b.fused = (b.cap % 64 == 0) && b.cap <= 0x7FFFFFFFull && step_launch_enabled();
    uint64_t swords = chr_propagate_scratch_words(chunk_cap);
    if (b.fused) swords = std::max<uint64_t>(swords, 16 + mask_scan_words(nphotons) + 16);
    const size_t qbytes = ((size_t)nphotons + 1) * 4;
    // split path: hits, ray counter, binning keys/order/histogram
    const size_t hbytes = b.fused ? (size_t)nphotons * 24 + 128 + 256 + 512 + sort_temp_bytes16(nphotons) : 0;
    // split path: ray records, queue order + walk order (FlatCtx::rays / rays_walk)
    const size_t rbytes = b.fused ? (size_t)nphotons * 64 + 512 : 0;
    const size_t base_bytes = 2 * qbytes + swords * 4 + 64 + hbytes + rbytes;
    const size_t mbytes = tail_masks ? ((size_t)nphotons + 63) / 64 * 8 + 512 : 0;
    void *buf = nullptr;
    int rc = scratch_get(base_bytes + mbytes, &buf, ctx);
    if (rc) return rc;
    b.q[0] = (uint32_t *)buf;
    b.q[1] = b.q[0] + (nphotons + 1);
    b.scratch = (uint32_t *)(((uintptr_t)(b.q[1] + nphotons + 1) + 15) & ~(uintptr_t)15);
    b.hits = b.fused ? (int2 *)(((uintptr_t)(b.scratch + swords) + 15) & ~(uintptr_t)15) : nullptr;
    // radix-sort space after [hits][next+pad][keys][order][hist][walk hist]
    b.sort_space = b.fused ? (uint32_t *)(((uintptr_t)((uint32_t *)(b.hits + nphotons) + 16 + 2 * (size_t)nphotons +
                                                       64) + 255) & ~(uintptr_t)255) : nullptr;
    b.tail_masks = tail_masks ? (unsigned long long *)(((uintptr_t)buf + base_bytes + 255) & ~(uintptr_t)255) : nullptr;
    if ((rc = pinned_words(&b.pinned, ctx))) return rc;
    if (b.fused && (rc = flat_get(nphotons, b.fc, ctx))) return rc;
    if (b.fused) {
        b.fc.rays = (uint4 *)(((uintptr_t)buf + 2 * qbytes + swords * 4 + 64 + hbytes + 255) & ~(uintptr_t)255);
        b.fc.rays_walk = b.fc.rays + 2 * (size_t)nphotons;
    }
    return CHR_OK;
}

// queues (photon.py:242-250: clones interleaved, q[1] header = 1), step counters, flat-walk control words
// (done: the device-driven slot loop's done flag, zeroed too)
static int prop_start(const PropBufs &b, uint32_t nphotons, uint32_t true_nphotons, uint32_t ncopies, hipStream_t stream,
                      uint32_t *done = nullptr) {
    ZeroWords z{{b.fused ? b.fc.ctl : nullptr, b.scratch, done}, {32u, 16u, 1u}};
    hipLaunchKernelGGL(init_queue_kernel, dim3(grid_for(nphotons)), dim3(BLOCK), 0, stream, b.q[0], b.q[1], nphotons,
                       true_nphotons, ncopies, z);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

// grow a slot event list to n events
static int grow_events(std::vector<hipEvent_t> &v, size_t n) {
    while (v.size() < n) {
        hipEvent_t e;
        CHR_HIP_CHECK(hipEventCreate(&e));
        v.push_back(e);
    }
    return CHR_OK;
}

// How device_slots runs a propagate besides its buffers.
struct SlotRun {
    std::vector<hipEvent_t> *events = nullptr;   // SLOT_EVENTS per slot (grown here)
    hipStream_t tstream = nullptr;     // tail kernels go there (chr_propagate_batches; nullptr: on the stream)
    hipEvent_t rng_ready = nullptr;    // the first RNG use waits for it
    hipEvent_t prefix_done = nullptr;  // slot 0's prefix was queued by queue_prefix and ends with this event
    int ctx = 0;
};

// Device-driven steps: every slot's kernels read the queue length from the
// queue header and the head kernel applies the nsteps policy, so the host
// queues slot k + 1 while slot k runs and only waits (on slot k - 1's event,
// already done by then) to learn when the tail has run -- no survivor-count
// round trip between steps.  Same launches, same results.  *k_out = slots
// queued, *ctl_out = their [mode, length] words.
static int device_slots(const chr_geometry *g, const chr_photons *ph, uint32_t nphotons, uint32_t *rng, uint32_t nslots,
                        int32_t ntpb, int32_t max_steps, int32_t use_weights, int32_t scatter_first, PropBufs &b,
                        const SlotRun &run, hipStream_t stream, uint32_t **ctl_out, int *k_out) {
    const uint32_t tail_below = (uint32_t)ntpb * 16 * 8;   // photon.py:261-264
    uint32_t *ctl = nullptr;
    int rc = slot_ctl_get(2 * (size_t)max_steps + 8, &ctl, run.ctx);
    if (rc) return rc;
    uint32_t *done = ctl + 2 * (size_t)max_steps;
    if (!run.prefix_done) CHR_HIP_CHECK(hipMemsetAsync(done, 0, 4, stream));
    b.fc.enrol_next = true;
    uint32_t *ring = b.pinned + 64;   // (mode, n) of recent slots, 32 entries (written by each slot's head kernel)
    // slot k + 1's head runs at the end of slot k's scan (no head dispatch per slot)
    const bool fold = true;
    std::vector<hipEvent_t> &events = *run.events;
    uint32_t n_ub = nphotons;
    int k = 0, cur = 0;
    bool stop = false;
    while (k < max_steps && !stop) {
        if ((rc = grow_events(events, SLOT_EVENTS * (size_t)(k + 1)))) return rc;
        hipEvent_t *ev = events.data() + SLOT_EVENTS * (size_t)k;
        SlotCtl sc{ctl + 2 * (size_t)k, ctl + 2 * (size_t)k + 1, done, nphotons, max_steps - k, tail_below};
        sc.tail_stream = run.tstream;
        sc.tail_masks = b.tail_masks;
        const int timing = slot_timing();
        sc.evt_tail0 = timing == 2 ? ev[5] : nullptr;
        sc.evt_tail1 = timing == 2 ? ev[6] : nullptr;
        sc.rng_ready = k == 0 ? run.rng_ready : nullptr;
        sc.ctx = run.ctx;
        sc.host_ring = ring + 2 * (k % 32);   // written by the slot's head kernel (slot 0 of a batch: its prefix's)
        sc.fold_head = fold;
        if (fold && k + 1 < max_steps)
            sc.next_head = HeadNext{ctl + 2 * (size_t)(k + 1), ctl + 2 * (size_t)(k + 1) + 1, done, nullptr,
                                    ring + 2 * ((k + 1) % 32), tail_below, nphotons, max_steps - k - 1, use_weights};
        if (k == 0 && run.prefix_done) {
            sc.phase = PHASE_REST;
            sc.prefix_done = run.prefix_done;
            sc.ev_rest0 = timing == 2 ? ev[7] : nullptr;
        }
        bool split = false;
        // ev[2] (before the slot's trace) is always recorded: the host's and the tail
        // stream's sync point for the slot (its head has run); the end-of-slot event ev[4]
        // only with every slot event (CHR_SLOT_TIMING=1), else once after the last slot
        rc = launch_step(g, ph, rng, nslots, (uint32_t)b.cap, n_ub, b.q[cur] + 1, b.q[cur ^ 1], 1, use_weights,
                         scatter_first, b.scratch, stream, timing == 2 ? ev[0] : nullptr, timing == 2 ? ev[1] : nullptr,
                         b.hits, b.sort_space, k == 0, ev[2], timing ? ev[3] : nullptr, &split, &b.fc, &sc);
        if (rc) return rc;
        if (timing == 2) CHR_HIP_CHECK(hipEventRecord(ev[4], stream));
        cur ^= 1;
        scatter_first = 0;
        if (k >= 1) {   // slot k - 1's head has run (its mode is known): is there a slot k + 1?
            CHR_HIP_CHECK(hipEventSynchronize(events[SLOT_EVENTS * (size_t)(k - 1) + (timing == 2 ? 4 : 2)]));
            const uint32_t m = ring[2 * ((k - 1) % 32)], nk = ring[2 * ((k - 1) % 32) + 1];
            if (m != STEP_ONE) stop = true;   // the tail ran or the queue emptied: slot k is idle
            else n_ub = nk;                   // later queues are no longer
        }
        k++;
    }
    if (k > 0 && slot_timing() != 2)   // the end of the last slot (the batch's read-back waits for it)
        CHR_HIP_CHECK(hipEventRecord(events[SLOT_EVENTS * (size_t)(k - 1) + 4], stream));
    *ctl_out = ctl;
    *k_out = k;
    return CHR_OK;
}

// per-slot statistics of a finished device-driven propagate (h: [mode, length]
// per slot); prefixed: slot 0 ran as prefix + rest (chr_propagate_batches)
static int slot_stats(chr_propagate_stats &st, const uint32_t *h, int k, const std::vector<hipEvent_t> &events,
                      bool tail_stream, bool prefixed = false) {
    const int timing = slot_timing();
    for (int j = 0; j < k; ++j) {
        const uint32_t m = h[2 * j], nj = h[2 * j + 1];
        const hipEvent_t *ev = events.data() + SLOT_EVENTS * (size_t)j;
        float ms = 0.0f;
        if (timing < 2) {   // (CHR_SLOT_TIMING) counts only, and the trace launches' times
            if (m == STEP_IDLE) continue;
            st.launches++;
            st.steps_run++;
            if (m == STEP_ONE) {
                if (timing == 1) CHR_HIP_CHECK(hipEventElapsedTime(&ms, ev[2], ev[3]));
                st.trace_ms += ms;
                if (st.trace_ms_n < CHR_TRACE_MS_MAX) {
                    st.trace_launch_rays[st.trace_ms_n] = nj;
                    st.trace_launch_ms[st.trace_ms_n++] = ms;
                }
                st.trace_launches++;
                st.trace_rays += nj;
            } else {
                st.tail_photons += nj;
            }
            continue;
        }
        if (j == 0 && prefixed) {   // the prefix on its stream (binning, walk), the rest after it on the batch stream
            float ms2 = 0.0f;
            CHR_HIP_CHECK(hipEventElapsedTime(&ms, ev[0], ev[3]));    // head, binning, trace
            CHR_HIP_CHECK(hipEventElapsedTime(&ms2, ev[7], ev[1]));   // shade, scan, scatter
            ms += ms2;
        } else {
            CHR_HIP_CHECK(hipEventElapsedTime(&ms, ev[0], ev[1]));
        }
        st.kernel_ms += ms;
        if (m == STEP_IDLE) continue;
        st.launches++;
        st.steps_run++;
        if (m == STEP_ONE) {
            CHR_HIP_CHECK(hipEventElapsedTime(&ms, ev[2], ev[3]));
            st.trace_ms += ms;
            if (st.trace_ms_n < CHR_TRACE_MS_MAX) {
                st.trace_launch_rays[st.trace_ms_n] = nj;
                st.trace_launch_ms[st.trace_ms_n++] = ms;
            }
            st.trace_launches++;
            st.trace_rays += nj;
        } else {
            if (tail_stream) {
                CHR_HIP_CHECK(hipEventElapsedTime(&ms, ev[5], ev[6]));
                st.kernel_ms += ms;
            }
            st.tail_ms += ms;
            st.tail_photons += nj;
        }
    }
    return CHR_OK;
}

// device counters of a propagate -> pinned words [2] overflows, [4..17] walk
// counters, [20..36] flat-walk and tail diagnostics (fused path)
static int counter_readback(const PropBufs &b, hipStream_t s) {
    CHR_HIP_CHECK(hipMemcpyAsync(b.pinned + 2, b.scratch, 4, hipMemcpyDeviceToHost, s));
    CHR_HIP_CHECK(hipMemcpyAsync(b.pinned + 4, b.scratch + 2, 56, hipMemcpyDeviceToHost, s));
    if (b.fused) CHR_HIP_CHECK(hipMemcpyAsync(b.pinned + 20, b.fc.ctl + 3, 68, hipMemcpyDeviceToHost, s));
    return CHR_OK;
}

static void counter_stats(chr_propagate_stats &st, const PropBufs &b) {
    const uint32_t *pinned = b.pinned;
    st.stack_overflows = pinned[2];
    st.flat_walks = b.fused ? pinned[20] : 0u;
    st.flat_walks_whole = b.fused ? pinned[21] : 0u;
    if (b.fused) {
        uint64_t key;
        std::memcpy(&key, pinned + 23, 8);
        st.tail_max_steps = pinned[22];
        st.tail_max_cycles = key >> 16;
        st.tail_slowest_steps = (uint32_t)(key & 0xFFFFu);
        uint64_t lp[6];
        std::memcpy(lp, pinned + 25, 48);   // ctl[8..19]
        st.tail_long_walk_ticks = lp[0];
        st.tail_long_ticks = lp[1];
        st.tail_long_walk_iterations = lp[2];
        st.tail_long_steps = lp[3];
        st.tail_long_photons = (uint32_t)lp[4];
        st.tail_long_paired_steps = (uint32_t)lp[5];
    }
    uint64_t c[7];
    std::memcpy(c, pinned + 4, 56);
    st.wave_fill_cycles = c[5];
    st.wave_step_cycles = c[6];
    st.nodes_visited = c[0];
    st.triangles_tested = c[1];
    st.traversals = c[2];
    st.wave_node_steps = c[3];
    st.wave_triangle_steps = c[4];
}

static int check_propagate_args(const char *fn, const chr_geometry *g, const chr_photons *ph, uint32_t nphotons,
                                uint32_t true_nphotons, uint32_t ncopies, const uint32_t *d_rng_states,
                                uint32_t rng_nslots, int32_t ntpb, int32_t max_blocks, int32_t max_steps) {
    if (!g || !photons_ok(ph) || !d_rng_states) return chr::fail(CHR_ERR_INVALID, "%s: null argument", fn);
    if (ntpb <= 0 || max_blocks <= 0) return chr::fail(CHR_ERR_INVALID, "%s: bad launch shape", fn);
    // the slot-control words are sized by max_steps (device_slots, queue_prefix)
    if (max_steps < 0) return chr::fail(CHR_ERR_INVALID, "%s: max_steps must be >= 0 (got %d)", fn, max_steps);
    if ((uint64_t)ntpb * (uint64_t)max_blocks > rng_nslots)
        return chr::fail(CHR_ERR_INVALID, "%s: rng_states must hold nthreads_per_block*max_blocks=%lld states (have %u)",
                         fn, (long long)ntpb * max_blocks, rng_nslots);
    if (ncopies == 0 || (uint64_t)true_nphotons * ncopies != nphotons)
        return chr::fail(CHR_ERR_INVALID, "%s: nphotons != true_nphotons*ncopies", fn);
    if (nphotons > 0x7FFFFFFFu) return chr::fail(CHR_ERR_INVALID, "%s: more than 2^31-1 photons", fn);
    return CHR_OK;
}

static bool device_steps_ok(const chr_geometry *g, const PropBufs &b) {
    const StepVariant sv = select_step_variant(g);
    return b.fused && !trace_steps() && !host_steps_forced() && sv.trace && sv.tail;   // a slot queues both
}

extern "C" int chr_propagate(const chr_geometry *g, const chr_photons *ph, uint32_t nphotons, uint32_t true_nphotons,
                             uint32_t ncopies, uint32_t *d_rng_states, uint32_t rng_nslots, int32_t ntpb,
                             int32_t max_blocks, int32_t max_steps, int32_t use_weights, int32_t scatter_first,
                             chr_propagate_stats *stats, void *vstream) {
    CHR_TRY(check_propagate_args("chr_propagate", g, ph, nphotons, true_nphotons, ncopies, d_rng_states, rng_nslots,
                                 ntpb, max_blocks, max_steps));
    chr_propagate_stats st{};
    // max_steps == 0: the reference's step loop (photon.py:255) runs no launch
    if (nphotons == 0 || max_steps == 0) {
        st.final_alive = max_steps == 0 ? nphotons : 0u;
        if (stats) *stats = st;
        return CHR_OK;
    }
    if (walks_reference_bvh(g)) CHR_TRY(chr::geometry_ref_nodes(g));
    hipStream_t stream = (hipStream_t)vstream;
    PropBufs b;
    int rc = prop_bufs(nphotons, ntpb, max_blocks, 0, false, b);
    if (rc) return rc;
    const uint64_t cap = b.cap;
    const uint32_t chunk_cap = (uint32_t)std::min<uint64_t>(cap, nphotons);
    const bool fused = b.fused;
    uint32_t *const *q = b.q;
    uint32_t *scratch = b.scratch, *pinned = b.pinned;
    int2 *hits = b.hits;
    uint32_t *sort_space = b.sort_space;
    FlatCtx &fc = b.fc;
    if ((rc = prop_start(b, nphotons, true_nphotons, ncopies, stream))) return rc;
    fc.enrol_next = fused;
    const size_t max_chunks = fused ? 2 : (nphotons + chunk_cap - 1) / chunk_cap;   // fused: step + its walk
    std::vector<hipEvent_t> *evp = nullptr;
    if ((rc = timing_events(2 * max_chunks, &evp))) return rc;
    std::vector<hipEvent_t> &events = *evp;
    double kernel_ms = 0.0, trace_ms = 0.0;
    bool split_step = false, tail_step = false;
    int64_t n_launch = 0;   // queue length of the launch being collected
    auto collect = [&](size_t nchunks) -> int {
        for (size_t c = 0; c < nchunks; ++c) {
            float ms = 0.0f;
            CHR_HIP_CHECK(hipEventElapsedTime(&ms, events[2 * c], events[2 * c + 1]));
            kernel_ms += ms;
            if (tail_step) st.tail_ms += ms;
        }
        if (fused && split_step) {
            float ms = 0.0f;
            CHR_HIP_CHECK(hipEventElapsedTime(&ms, events[2], events[3]));
            trace_ms += ms;
            if (st.trace_ms_n < CHR_TRACE_MS_MAX) {
                st.trace_launch_rays[st.trace_ms_n] = (uint32_t)n_launch;
                st.trace_launch_ms[st.trace_ms_n++] = ms;
            }
        }
        return CHR_OK;
    };
    int cur = 0;
    int64_t n = nphotons;
    int step = 0;
    const bool device_steps = device_steps_ok(g, b);
    if (device_steps) {
        uint32_t *ctl = nullptr;
        int k = 0;
        SlotRun run;
        if ((rc = timing_events(0, &run.events))) return rc;
        if ((rc = device_slots(g, ph, nphotons, d_rng_states, rng_nslots, ntpb, max_steps, use_weights, scatter_first,
                               b, run, stream, &ctl, &k)))
            return rc;
        CHR_HIP_CHECK(hipStreamSynchronize(stream));
        st.host_syncs = 1;
        std::vector<uint32_t> h(2 * (size_t)k);
        CHR_HIP_CHECK(hipMemcpy(h.data(), ctl, 8 * (size_t)k, hipMemcpyDeviceToHost));
        if ((rc = timing_events(0, &evp))) return rc;
        if ((rc = slot_stats(st, h.data(), k, *evp, false))) return rc;
        step = max_steps;   // as the host loop: it leaves early only on an empty queue
        n = 0;
    }
    while (!device_steps && step < max_steps) {
        const int nsteps = (n < (int64_t)ntpb * 16 * 8 || use_weights) ? max_steps - step : 1;   // photon.py:261-264
        const int64_t n_prev = n;
        n_launch = n;
        tail_step = nsteps > 1;
        if (tail_step) st.tail_photons += (uint32_t)n;
        size_t nchunks = 0;
        if (fused) {
            rc = launch_step(g, ph, d_rng_states, rng_nslots, (uint32_t)cap, (uint32_t)n, q[cur] + 1, q[cur ^ 1],
                             nsteps, use_weights, scatter_first, scratch, stream, events[0], events[1], hits,
                             sort_space, step == 0, events[2], events[3], &split_step, &fc);
            if (rc) return rc;
            st.launches++;
            nchunks = 1;
            if (split_step) {
                st.trace_launches++;
                st.trace_rays += (uint64_t)n;
            }
        } else {
            int64_t first = 0;
            while (first < n) {
                // chunk_iterator (tools.py:159-180)
                const int64_t left = n - first;
                int64_t blocks = left / ntpb + (left % ntpb != 0);
                if (blocks > max_blocks) blocks = max_blocks;
                const int64_t count = std::min<int64_t>(left, blocks * ntpb);
                rc = launch_chunk(g, ph, d_rng_states, rng_nslots, (int32_t)first, (int32_t)count, q[cur] + 1,
                                  q[cur ^ 1], nsteps, use_weights, scatter_first, scratch, stream, events[2 * nchunks],
                                  events[2 * nchunks + 1]);
                if (rc) return rc;
                st.launches++;
                nchunks++;
                first += count;
            }
        }
        st.steps_run++;
        step += nsteps;
        scatter_first = 0;
        if (step < max_steps) {
            cur ^= 1;
            // read the survivor count (photon.py:284) and reset the other header
            CHR_HIP_CHECK(hipMemcpyAsync(pinned, q[cur], 4, hipMemcpyDeviceToHost, stream));
            CHR_HIP_CHECK(hipStreamSynchronize(stream));
            st.host_syncs++;
            if ((rc = collect(nchunks))) return rc;
            nchunks = 0;
            n = (int64_t)pinned[0] - 1;
            if (trace_steps()) {
                fprintf(stderr, "chr_propagate: step %d nsteps %d -> %lld alive\n", step, nsteps, (long long)n);
                if (nsteps == 1 && hits) {   // walk-cost histogram of a counting trace variant (zeros otherwise)
                    uint32_t wh[34];
                    CHR_HIP_CHECK(hipMemcpy(wh, (uint32_t *)(hits + n_prev) + 16 + 2 * (size_t)n_prev, sizeof(wh),
                                            hipMemcpyDeviceToHost));
                    fprintf(stderr, "  walk cost (nodes+triangles) log2 histogram:");
                    for (int b = 0; b < 32; ++b) if (wh[b]) fprintf(stderr, " [%u,%u):%u", 1u << b, 2u << b, wh[b]);
                    fprintf(stderr, "\n  worst walk: cost %u photon %u\n", wh[33], wh[32]);
                }
            }
            pinned[1] = 1;
            CHR_HIP_CHECK(hipMemcpyAsync(q[cur ^ 1], pinned + 1, 4, hipMemcpyHostToDevice, stream));
            if (n == 0) break;
        }
        if (nchunks) {   // last step (no survivor read-back): drain before collecting
            CHR_HIP_CHECK(hipStreamSynchronize(stream));
            st.host_syncs++;
            if ((rc = collect(nchunks))) return rc;
        }
    }
    if ((rc = counter_readback(b, stream))) return rc;
    CHR_HIP_CHECK(hipStreamSynchronize(stream));
    counter_stats(st, b);
    st.kernel_ms += kernel_ms;
    st.trace_ms += trace_ms;
    st.final_alive = (step < max_steps) ? (uint32_t)n : 0u;
    if (stats) *stats = st;
    return CHR_OK;
}

// the streams of chr_propagate_batches (per thread and device; non-blocking:
// no implicit ordering with the legacy default stream): tails, and the
// prefixes (first-step queueing, binning and walk) of the batches ahead
static int batch_streams_get(hipStream_t *tail, hipStream_t *prefix) {
    static thread_local hipStream_t ts[16][2] = {};
    int dev = 0;
    CHR_HIP_CHECK(hipGetDevice(&dev));
    hipStream_t *s = ts[dev & 15];
    if (!s[0]) {   // the tails are the critical path: the highest stream priority
        int least = 0, greatest = 0;
        CHR_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
        CHR_HIP_CHECK(hipStreamCreateWithPriority(&s[0], hipStreamNonBlocking, greatest));
        CHR_HIP_CHECK(hipStreamCreateWithPriority(&s[1], hipStreamNonBlocking, least));
    }
    *tail = s[0];
    *prefix = s[1];
    return CHR_OK;
}

// Host-side resources of one batch of a chr_propagate_batches call: its slot
// events, its prefix / done events, pinned words ([0..63] counters read back,
// [64..127] the slot ring, [128..] the slot control words).  Per thread and
// device, reused across calls (every call drains before it returns).
struct BatchHost {
    std::vector<hipEvent_t> ev;
    hipEvent_t prefix_done = nullptr, done = nullptr;
    uint32_t *pinned = nullptr;
    size_t words = 0;
};
static int batch_host_get(size_t nb, size_t words, std::vector<BatchHost> **out) {
    static thread_local std::vector<BatchHost> pool[16];
    int dev = 0;
    CHR_HIP_CHECK(hipGetDevice(&dev));
    std::vector<BatchHost> &v = pool[dev & 15];
    if (v.size() < nb) v.resize(nb);
    for (size_t i = 0; i < nb; ++i) {
        BatchHost &b = v[i];
        if (!b.prefix_done) CHR_HIP_CHECK(hipEventCreateWithFlags(&b.prefix_done, hipEventDisableTiming));
        if (!b.done) CHR_HIP_CHECK(hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
        if (b.words < words) {
            if (b.pinned) CHR_HIP_CHECK(hipHostFree(b.pinned));
            b.pinned = nullptr;
            CHR_HIP_CHECK(hipHostMalloc((void **)&b.pinned, words * 4, hipHostMallocDefault));
            b.words = words;
        }
    }
    *out = &v;
    return CHR_OK;
}

static bool ranges_overlap(const void *a, size_t na, const void *b, size_t nb) {
    const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
    return a && b && x < y + nb && y < x + na;
}
// whether two batches share any photon array (then the later one waits for the earlier one)
static bool photons_alias(const chr_photons *a, uint32_t na, const chr_photons *b, uint32_t nb) {
    const void *pa[9] = {a->d_pos, a->d_dir, a->d_pol, a->d_wavelengths, a->d_t, a->d_weights, a->d_flags,
                         a->d_last_hit_triangles, a->d_evidx};
    const void *pb[9] = {b->d_pos, b->d_dir, b->d_pol, b->d_wavelengths, b->d_t, b->d_weights, b->d_flags,
                         b->d_last_hit_triangles, b->d_evidx};
    const size_t w[9] = {12, 12, 12, 4, 4, 4, 4, 4, 4};
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j)
            if (ranges_overlap(pa[i], w[i] * na, pb[j], w[j] * nb)) return true;
    return false;
}

// The RNG-free part of a propagate's first slot on stream ps: queues, counters,
// the head kernel, flat-walk classification, direction binning and the BVH walk
// (launch_step PHASE_PREFIX), ending with prefix_done.
// Measured and removed: queueing the prefixes of later batches
// earlier (r02 ab_lookahead: one batch ahead 417.3, two 378.2 against 416.8 M/s),
// the next batch's prefix once the running one is down to few photons (r02
// ab_prefix_trigger, 392 against 428 M/s), its binning early (r03 ab5, 412.0
// against 425.1 M/s), and the prefix walk on a fraction of the grid (r03 ab4):
// a walk started beside the running batch's late steps or its tail slows them
// more than the overlap gains.
static int queue_prefix(const chr_geometry *g, const chr_photons *ph, uint32_t nphotons, uint32_t true_nphotons,
                        uint32_t ncopies, uint32_t *rng, uint32_t nslots, int32_t ntpb, int32_t max_steps,
                        int32_t use_weights, int32_t scatter_first, PropBufs &b, int ctx,
                        std::vector<hipEvent_t> &events, hipEvent_t prefix_done, hipStream_t ps) {
    uint32_t *ctl = nullptr;
    CHR_TRY(slot_ctl_get(2 * (size_t)max_steps + 8, &ctl, ctx));
    uint32_t *done = ctl + 2 * (size_t)max_steps;
    CHR_TRY(prop_start(b, nphotons, true_nphotons, ncopies, ps, done));
    b.fc.enrol_next = true;
    CHR_TRY(grow_events(events, SLOT_EVENTS));
    SlotCtl sc{ctl, ctl + 1, done, nphotons, max_steps, (uint32_t)ntpb * 16 * 8};
    sc.phase = PHASE_PREFIX;
    sc.ctx = ctx;
    sc.prefix_done = prefix_done;
    sc.host_ring = b.pinned + 64;   // ring entry 0 (device_slots' slot 0): this head is slot 0's
    hipEvent_t *ev = events.data();
    const int timing = slot_timing();
    return launch_step(g, ph, rng, nslots, (uint32_t)b.cap, nphotons, b.q[0] + 1, b.q[1], 1, use_weights,
                       scatter_first, b.scratch, ps, timing == 2 ? ev[0] : nullptr, ev[1], b.hits, b.sort_space, true,
                       ev[2], timing ? ev[3] : nullptr, nullptr,
                       &b.fc, &sc);
}

static int propagate_batches(const chr_geometry *g, const chr_photons *phs, const uint32_t *nphotons,
                             const uint32_t *true_nphotons, const uint32_t *ncopies, uint32_t nbatch,
                             uint32_t *d_rng_states, uint32_t rng_nslots, int32_t ntpb, int32_t max_blocks,
                             int32_t max_steps, int32_t use_weights, int32_t scatter_first, chr_propagate_stats *stats,
                             void *vstream) {
    if (nbatch && (!phs || !nphotons || !true_nphotons || !ncopies))
        return chr::fail(CHR_ERR_INVALID, "chr_propagate_batches: null argument");
    for (uint32_t i = 0; i < nbatch; ++i)
        CHR_TRY(check_propagate_args("chr_propagate_batches", g, phs + i, nphotons[i], true_nphotons[i], ncopies[i],
                                     d_rng_states, rng_nslots, ntpb, max_blocks, max_steps));
    hipStream_t stream = (hipStream_t)vstream;
    if (stats)
        for (uint32_t i = 0; i < nbatch; ++i) {
            stats[i] = chr_propagate_stats{};
            if (max_steps == 0) stats[i].final_alive = nphotons[i];
        }
    if (max_steps == 0) return CHR_OK;   // as max_steps == 0 propagate calls: no launch
    // the non-empty batches, in order
    std::vector<uint32_t> idx;
    uint32_t max_n = 0;
    for (uint32_t i = 0; i < nbatch; ++i)
        if (nphotons[i]) { idx.push_back(i); max_n = std::max(max_n, nphotons[i]); }
    if (idx.empty()) return CHR_OK;
    if (walks_reference_bvh(g)) CHR_TRY(chr::geometry_ref_nodes(g));
    PropBufs probe;
    probe.cap = (uint64_t)ntpb * max_blocks;
    probe.fused = (probe.cap % 64 == 0) && probe.cap <= 0x7FFFFFFFull && step_launch_enabled();
    if (idx.size() == 1 || !device_steps_ok(g, probe)) {   // nothing to overlap: one propagate after the other
        for (uint32_t i : idx)
            CHR_TRY(chr_propagate(g, phs + i, nphotons[i], true_nphotons[i], ncopies[i], d_rng_states, rng_nslots,
                                  ntpb, max_blocks, max_steps, use_weights, scatter_first, stats ? stats + i : nullptr,
                                  vstream));
        return CHR_OK;
    }
    hipStream_t ts = nullptr, ps = nullptr;
    CHR_TRY(batch_streams_get(&ts, &ps));
    const size_t nb = idx.size();
    std::vector<BatchHost> *pool = nullptr;
    CHR_TRY(batch_host_get(nb, 128 + 2 * (size_t)max_steps + 8, &pool));
    std::vector<BatchHost> &bh = *pool;
    // every context sized for the largest batch up front: no buffer is
    // reallocated while an earlier batch may still use it
    PropBufs bufs[NCTX];
    for (int c = 0; c < NCTX && c < (int)nb; ++c) {
        CHR_TRY(prop_bufs(max_n, ntpb, max_blocks, c, true, bufs[c]));
        uint32_t *ctl = nullptr;
        CHR_TRY(slot_ctl_get(2 * (size_t)max_steps + 8, &ctl, c));
        const int cus = device_cus();
        const StepVariant sv = select_step_variant(g);
        const uint64_t tb = (uint64_t)sv.trace_block;
        const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)cus * 4 * sv.trace_waves * 64 / tb,
                                                                          ((uint64_t)max_n + tb - 1) / tb));
        uint2 *spill = nullptr;
        CHR_TRY(walk_stack_get((size_t)WIDE_STACK * blocks * tb * sizeof(uint2), &spill, c));
    }
    // the photon inputs were written on the caller's stream
    std::vector<hipEvent_t> *entry_ev = nullptr;
    CHR_TRY(timing_events(1, &entry_ev, 1));
    CHR_HIP_CHECK(hipEventRecord((*entry_ev)[0], stream));
    CHR_HIP_CHECK(hipStreamWaitEvent(ps, (*entry_ev)[0], 0));
    // batch j's prefix is queued when batch j starts (after batch j - 1's slots, so
    // it runs beside that batch's tail)
    auto prefix = [&](size_t j) -> int {
        const uint32_t i = idx[j];
        const int c = (int)(j % NCTX);
        if (j >= (size_t)NCTX) CHR_HIP_CHECK(hipStreamWaitEvent(ps, bh[j - NCTX].done, 0));   // the context is free
        for (size_t e = j >= (size_t)NCTX ? j - NCTX + 1 : 0; e < j; ++e)   // shared photon arrays: after that batch
            if (photons_alias(phs + i, nphotons[i], phs + idx[e], nphotons[idx[e]]))
                CHR_HIP_CHECK(hipStreamWaitEvent(ps, bh[e].done, 0));
        CHR_TRY(prop_bufs(nphotons[i], ntpb, max_blocks, c, true, bufs[c]));
        bufs[c].pinned = bh[j].pinned;
        return queue_prefix(g, phs + i, nphotons[i], true_nphotons[i], ncopies[i], d_rng_states, rng_nslots, ntpb,
                            max_steps, use_weights, scatter_first, bufs[c], c, bh[j].ev, bh[j].prefix_done, ps);
    };
    std::vector<int> slots(nb, 0);
    for (size_t j = 0; j < nb; ++j) {
        CHR_TRY(prefix(j));
        const uint32_t i = idx[j];
        const int c = (int)(j % NCTX);
        PropBufs &b = bufs[c];
        SlotRun run;
        run.events = &bh[j].ev;
        run.tstream = ts;
        run.rng_ready = j > 0 ? bh[j - 1].done : nullptr;   // the previous batch's tail advances the RNG slots
        run.prefix_done = bh[j].prefix_done;
        run.ctx = c;
        uint32_t *ctl = nullptr;
        CHR_TRY(device_slots(g, phs + i, nphotons[i], d_rng_states, rng_nslots, ntpb, max_steps, use_weights,
                             scatter_first, b, run, stream, &ctl, &slots[j]));
        // after the batch's last slot (and every tail before it on ts): read its counters back
        CHR_HIP_CHECK(hipStreamWaitEvent(ts, bh[j].ev[SLOT_EVENTS * (size_t)(slots[j] - 1) + 4], 0));
        CHR_HIP_CHECK(hipMemcpyAsync(bh[j].pinned + 128, ctl, 8 * (size_t)slots[j], hipMemcpyDeviceToHost, ts));
        CHR_TRY(counter_readback(b, ts));
        CHR_HIP_CHECK(hipEventRecord(bh[j].done, ts));
    }
    // the last batch's done event follows every earlier one on the tail stream
    CHR_HIP_CHECK(hipEventSynchronize(bh[nb - 1].done));
    for (size_t j = 0; j < nb; ++j) {
        chr_propagate_stats st{};
        CHR_TRY(slot_stats(st, bh[j].pinned + 128, slots[j], bh[j].ev, true, true));
        PropBufs view;
        view.fused = true;
        view.pinned = bh[j].pinned;
        counter_stats(st, view);
        st.host_syncs = 1;
        st.final_alive = 0;
        if (stats) stats[idx[j]] = st;
    }
    return CHR_OK;
}

extern "C" int chr_propagate_batches(const chr_geometry *g, const chr_photons *phs, const uint32_t *nphotons,
                                     const uint32_t *true_nphotons, const uint32_t *ncopies, uint32_t nbatch,
                                     uint32_t *d_rng_states, uint32_t rng_nslots, int32_t ntpb, int32_t max_blocks,
                                     int32_t max_steps, int32_t use_weights, int32_t scatter_first,
                                     chr_propagate_stats *stats, void *vstream) {
    const int rc = propagate_batches(g, phs, nphotons, true_nphotons, ncopies, nbatch, d_rng_states, rng_nslots, ntpb,
                                     max_blocks, max_steps, use_weights, scatter_first, stats, vstream);
    // a failure part-way leaves work queued on three streams: drain it, so no
    // buffer of this call is still in use when the caller frees or retries
    if (rc != CHR_OK) (void)hipDeviceSynchronize();
    return rc;
}

static int select_common(const chr_photons *ph, int32_t start, int32_t n, uint32_t state, const uint32_t *solid_map,
                         const int32_t *s2c, int mode, const chr_photons *out, int32_t *channels, uint32_t *count,
                         hipStream_t stream) {
    if (!count) return chr::fail(CHR_ERR_INVALID, "selection: null count");
    *count = 0;
    // an empty selection needs no photon arrays (a GPUPhotons of 0 photons, e.g. a
    // rank's empty shard of a batch, has none)
    if (n <= 0 && ph) return CHR_OK;
    if (!photons_ok(ph)) return chr::fail(CHR_ERR_INVALID, "selection: null argument");
    if (mode == 0 && (!solid_map || !s2c)) return chr::fail(CHR_ERR_INVALID, "hits: solid map / channel map missing");
    const uint32_t nwords = (uint32_t)((n + 63) / 64);
    void *buf;
    int rc = scratch_get((mask_scan_words((uint64_t)n) + 8) * 4 + 64, &buf);
    if (rc) return rc;
    uint32_t *cnt = (uint32_t *)buf;
    unsigned long long *masks = (unsigned long long *)((uint32_t *)buf + 8);
    uint32_t *offsets = (uint32_t *)buf + 8 + 2 * (size_t)nwords;
    uint32_t *bsums = offsets + nwords;
    const PhotonPtrs p = to_ptrs(ph);
    hipLaunchKernelGGL(flag_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, stream, p, start, n, state, solid_map, s2c, mode,
                       masks);
    launch_mask_scan(masks, nwords, offsets, bsums, nullptr, nullptr, cnt, stream);
    CHR_HIP_CHECK(hipGetLastError());
    uint32_t total = 0;
    CHR_HIP_CHECK(hipMemcpyAsync(&total, cnt, 4, hipMemcpyDeviceToHost, stream));
    CHR_HIP_CHECK(hipStreamSynchronize(stream));
    *count = total;
    if (out && total > 0) {
        if (!photons_ok(out)) return chr::fail(CHR_ERR_INVALID, "selection: output buffers missing");
        hipLaunchKernelGGL(copy_selected_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, stream, p, start, n, masks, offsets,
                           bsums, to_ptrs(out), channels, solid_map, s2c);
        CHR_HIP_CHECK(hipGetLastError());
        CHR_HIP_CHECK(hipStreamSynchronize(stream));
    }
    return CHR_OK;
}

extern "C" int chr_photon_hits(const chr_photons *ph, int32_t start_photon, int32_t nphotons, uint32_t detection_state,
                               const uint32_t *d_solid_map, const int32_t *d_solid_id_to_channel_index,
                               const chr_photons *d_out, int32_t *d_out_channels, uint32_t *nhits, void *stream) {
    return select_common(ph, start_photon, nphotons, detection_state, d_solid_map, d_solid_id_to_channel_index, 0, d_out,
                         d_out_channels, nhits, (hipStream_t)stream);
}

extern "C" int chr_select_photons(const chr_photons *ph, int32_t start_photon, int32_t nphotons, uint32_t target_flag,
                                  const chr_photons *d_out, uint32_t *nselected, void *stream) {
    return select_common(ph, start_photon, nphotons, target_flag, nullptr, nullptr, 1, d_out, nullptr, nselected,
                         (hipStream_t)stream);
}

extern "C" int chr_copy_photon_queue(const chr_photons *ph, int32_t first_photon, int32_t nphotons,
                                     const uint32_t *d_queue, const chr_photons *d_out, void *stream) {
    if (!photons_ok(ph) || !photons_ok(d_out) || !d_queue) return chr::fail(CHR_ERR_INVALID, "copy_queue: null argument");
    if (nphotons <= 0) return CHR_OK;
    hipLaunchKernelGGL(copy_queue_kernel, dim3(grid_for(nphotons)), dim3(BLOCK), 0, (hipStream_t)stream, to_ptrs(ph),
                       first_photon, nphotons, d_queue, to_ptrs(d_out));
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_photon_duplicate(const chr_photons *ph, int32_t first_photon, int32_t nphotons, int32_t copies,
                                    int32_t stride, void *stream) {
    if (!photons_ok(ph)) return chr::fail(CHR_ERR_INVALID, "duplicate: null argument");
    if (nphotons <= 0 || copies <= 0) return CHR_OK;
    hipLaunchKernelGGL(duplicate_kernel, dim3(grid_for(nphotons)), dim3(BLOCK), 0, (hipStream_t)stream, to_ptrs(ph),
                       first_photon, nphotons, copies, stride);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_kernel_info(int32_t which, chr_kernel_attr *out) {
    if (!out) return chr::fail(CHR_ERR_INVALID, "chr_kernel_info: null output");
    const void *fn = nullptr;
    const char *name = nullptr;
    switch (which) {
        case 0: fn = (const void *)trace_kernel<false, 6, 12, 4, 48>; name = "chr::trace_kernel<false,6,12,4,48>"; break;
        case 1: fn = (const void *)shade_kernel<3>; name = "chr::shade_kernel<3>"; break;
        case 2: fn = (const void *)propagate_tail_kernel<kTailWaves>; name = "chr::propagate_tail_kernel<2>"; break;
        case 3: fn = (const void *)propagate_step_kernel<8, 4, kWalk>; name = "chr::propagate_step_kernel<8,4,2006>"; break;
        default: return chr::fail(CHR_ERR_INVALID, "chr_kernel_info: unknown kernel %d", which);
    }
    hipFuncAttributes fa;
    CHR_HIP_CHECK(hipFuncGetAttributes(&fa, fn));
    out->private_bytes = fa.localSizeBytes;
    out->lds_bytes = fa.sharedSizeBytes;
    out->vgprs = fa.numRegs;
    out->max_threads = fa.maxThreadsPerBlock;
    std::snprintf(out->name, sizeof(out->name), "%s", name);
    return CHR_OK;
}

extern "C" int chr_distance_to_mesh(const chr_geometry *g, uint32_t n, const float *d_origin, const float *d_direction,
                                    float *d_distance, void *stream) {
    if (!g || !d_origin || !d_direction || !d_distance) return chr::fail(CHR_ERR_INVALID, "distance_to_mesh: null argument");
    if (n == 0) return CHR_OK;
    const bool wide = !walks_reference_bvh(g);
    if (!wide) CHR_TRY(chr::geometry_ref_nodes(g));
    hipLaunchKernelGGL(wide ? distance_kernel<true> : distance_kernel<false>, dim3(grid_for(n)), dim3(BLOCK), 0,
                       (hipStream_t)stream, (const DevGeom *)g->d_dev, n, d_origin, d_direction, d_distance,
                       (uint32_t *)nullptr);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

// Device profile counters (profile.h; profiler.py:217-262 device_fetch / device_reset)
extern "C" int chr_device_profile_enabled(void) {
#ifdef CHR_DEVICE_PROFILE
    return 1;
#else
    return 0;
#endif
}

extern "C" int chr_device_profile_reset(void *stream) {
#ifdef CHR_DEVICE_PROFILE
    void *calls = nullptr, *cycles = nullptr;
    CHR_HIP_CHECK(hipGetSymbolAddress(&calls, HIP_SYMBOL(chr::chr_prof_calls)));
    CHR_HIP_CHECK(hipGetSymbolAddress(&cycles, HIP_SYMBOL(chr::chr_prof_cycles)));
    CHR_HIP_CHECK(hipMemsetAsync(calls, 0, sizeof(unsigned long long) * CHR_PROF_COUNT, (hipStream_t)stream));
    CHR_HIP_CHECK(hipMemsetAsync(cycles, 0, sizeof(unsigned long long) * CHR_PROF_COUNT, (hipStream_t)stream));
    return CHR_OK;
#else
    (void)stream;
    return chr::fail(CHR_ERR_INVALID, "device profiling symbols not found: load libchroma_amd_prof.so "
                                      "(built with -DCHR_DEVICE_PROFILE=1; CHROMA_DEVICE_PROFILE=1)");
#endif
}

extern "C" int chr_device_profile_fetch(uint64_t *h_calls, uint64_t *h_cycles, int32_t n, uint32_t *clock_khz) {
#ifdef CHR_DEVICE_PROFILE
    if (!h_calls || !h_cycles || n < 0 || n > CHR_PROF_COUNT)
        return chr::fail(CHR_ERR_INVALID, "device_profile_fetch: bad arguments");
    CHR_HIP_CHECK(hipDeviceSynchronize());
    unsigned long long c[CHR_PROF_COUNT], y[CHR_PROF_COUNT];
    CHR_HIP_CHECK(hipMemcpyFromSymbol(c, HIP_SYMBOL(chr::chr_prof_calls), sizeof(c)));
    CHR_HIP_CHECK(hipMemcpyFromSymbol(y, HIP_SYMBOL(chr::chr_prof_cycles), sizeof(y)));
    for (int i = 0; i < n; ++i) { h_calls[i] = c[i]; h_cycles[i] = y[i]; }
    if (clock_khz) {
        int dev = 0, khz = 0;
        CHR_HIP_CHECK(hipGetDevice(&dev));
        CHR_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, dev));
        *clock_khz = (uint32_t)khz;
    }
    return CHR_OK;
#else
    (void)h_calls; (void)h_cycles; (void)n; (void)clock_khz;
    return chr::fail(CHR_ERR_INVALID, "device profiling symbols not found: load libchroma_amd_prof.so "
                                      "(built with -DCHR_DEVICE_PROFILE=1; CHROMA_DEVICE_PROFILE=1)");
#endif
}

extern "C" int chr_watch_set(uint32_t photon, const float *d_pos_array) {
#ifdef CHR_DEVICE_PROFILE
    const unsigned long long arr = (unsigned long long)d_pos_array;
    const uint32_t zero = 0u;
    CHR_HIP_CHECK(hipDeviceSynchronize());
    CHR_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(chr::chr_watch_pid), &photon, sizeof(photon)));
    CHR_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(chr::chr_watch_array), &arr, sizeof(arr)));
    CHR_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(chr::chr_watch_n), &zero, sizeof(zero)));
    return CHR_OK;
#else
    (void)photon; (void)d_pos_array;
    return chr::fail(CHR_ERR_INVALID, "photon watch: load libchroma_amd_prof.so (CHROMA_DEVICE_PROFILE=1)");
#endif
}

extern "C" int chr_watch_ray(const float *h_origin, uint32_t *h_events, uint32_t max_events, uint32_t *nevents) {
#ifdef CHR_DEVICE_PROFILE
    CHR_HIP_CHECK(hipDeviceSynchronize());
    if (h_origin) {   // arm: the walk of the ray with this origin (bit-exact) is logged
        const uint32_t on = 1u, zero = 0u;
        CHR_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(chr::chr_wray_o), h_origin, 3 * sizeof(float)));
        CHR_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(chr::chr_wev_n), &zero, sizeof(zero)));
        CHR_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(chr::chr_wray_on), &on, sizeof(on)));
        return CHR_OK;
    }
    if (!h_events || !nevents) return chr::fail(CHR_ERR_INVALID, "watch_ray: bad arguments");
    uint32_t n = 0;
    CHR_HIP_CHECK(hipMemcpyFromSymbol(&n, HIP_SYMBOL(chr::chr_wev_n), sizeof(n)));
    *nevents = n;
    uint32_t k = n < max_events ? n : max_events;
    if (k > chr::CHR_WEV_MAX) k = chr::CHR_WEV_MAX;
    if (k) CHR_HIP_CHECK(hipMemcpyFromSymbol(h_events, HIP_SYMBOL(chr::chr_wev_buf), sizeof(uint32_t) * 8 * k));
    return CHR_OK;
#else
    (void)h_origin; (void)h_events; (void)max_events; (void)nevents;
    return chr::fail(CHR_ERR_INVALID, "photon watch: load libchroma_amd_prof.so (CHROMA_DEVICE_PROFILE=1)");
#endif
}

extern "C" int chr_watch_fetch(uint32_t *h_out, uint32_t max_records, uint32_t *nrecords) {
#ifdef CHR_DEVICE_PROFILE
    if (!h_out || !nrecords) return chr::fail(CHR_ERR_INVALID, "watch_fetch: bad arguments");
    CHR_HIP_CHECK(hipDeviceSynchronize());
    uint32_t n = 0;
    CHR_HIP_CHECK(hipMemcpyFromSymbol(&n, HIP_SYMBOL(chr::chr_watch_n), sizeof(n)));
    *nrecords = n;
    uint32_t k = n < max_records ? n : max_records;
    if (k > chr::CHR_WATCH_MAX) k = chr::CHR_WATCH_MAX;
    if (k) CHR_HIP_CHECK(hipMemcpyFromSymbol(h_out, HIP_SYMBOL(chr::chr_watch_buf), sizeof(uint32_t) * k * chr::CHR_WATCH_WORDS));
    return CHR_OK;
#else
    (void)h_out; (void)max_records; (void)nrecords;
    return chr::fail(CHR_ERR_INVALID, "photon watch: load libchroma_amd_prof.so (CHROMA_DEVICE_PROFILE=1)");
#endif
}

namespace chr {
// chr_walk_lone_timing: walk_lone on one wave per workgroup (walker 0), or the
// pair walk on two (walker 1: wave 0 walks, wave 1 tests), each ray reps times;
// walker 2: the pair walk with a 2-poll handshake budget, so handshakes are lost
// (the tail kernel's recovery path: the walk again with walk_lone, no more
// pairing in the workgroup once aborted); walker 3: walk_up from an arbitrary node
// (ray r: node (r * 2654435761) mod nodes -- any start covers the tree once);
// walker 4: walk_up from the leaf node of a given record (8-word rays: + record);
// walker 5: the grouped walk's climb (walk_segment<0, UP>, one 64-lane segment) from
// walker 3's start; walker 7: walker 3 with the start node's chain read beforehand (the
// tail's prefetch)
__global__ __launch_bounds__(128) void walk_lone_timing_kernel(const DevGeom *__restrict__ gdev, const float *rays,
                                                               uint32_t n, uint32_t reps, uint32_t *out,
                                                               int32_t walker) {
    __shared__ uint32_t stacks[8 * TAIL_STACK * 2];
    __shared__ uint32_t tris[2 * TAIL_TRI];
    __shared__ uint32_t box_s[PB_WORDS];
    CHR_LDS uint32_t *box = (CHR_LDS uint32_t *)box_s;
    const DevGeom &g = *gdev;
    uint32_t overflow = 0;
    const TopNodes top{nullptr, 0u};
    if (threadIdx.x == 0) {
        box[PB_STATE] = PS_IDLE;
        box[PB_ABORT] = 0u;
    }
    __syncthreads();
    if (threadIdx.x >= 64) {   // the tester wave (walkers 1, 2), else idle
        if (walker == 0 || walker >= 3) return;
        while (true) {
            uint32_t st = PS_IDLE;
            for (uint32_t i = 0; i < PAIR_SPIN_MAX * 8u; ++i) {
                st = lds_ld(box + PB_STATE);
                if (st == PS_REQ || st == PS_EXIT) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if (st != PS_REQ) return;
            uint32_t old = 0;
            if (threadIdx.x == 64) old = atomicCAS(&box_s[PB_STATE], PS_REQ, PS_TAKEN);
            if ((uint32_t)__builtin_amdgcn_readfirstlane((int)old) != PS_REQ) continue;
            lds_acquire();
            walk_pair_tester(g, box, (CHR_LDS uint32_t *)tris, walker == 2 ? 2u : PAIR_SPIN_MAX);
        }
    }
    for (uint32_t r = blockIdx.x; r < n; r += gridDim.x) {
        const float *ry = rays + (walker == 4 ? 8 : 7) * (size_t)r;
        const V3 o = v3(ry[0], ry[1], ry[2]), d = v3(ry[3], ry[4], ry[5]);
        const uint32_t last = __float_as_uint(ry[6]);
        uint32_t start = (uint32_t)(((unsigned long long)r * 2654435761ull) % g.nwnodes);
        if (walker == 4) start = gld(reinterpret_cast<const uint32_t *>(g.wtri + 4 * (size_t)__float_as_uint(ry[7])) + 15);
        for (uint32_t k = 0; k < reps; ++k) {
            float sd;
            uint32_t it = 0;
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
            bool lost = false;
            const bool pair = (walker == 1 || walker == 2) && lds_ld(box + PB_ABORT) == 0u;
            uint32_t pc = 0xFFFFFFFFu, pp = 0xFFFFFFFFu;
            if (walker == 7) {
                const uint32_t *cw = reinterpret_cast<const uint32_t *>(g.wnodes + (size_t)g.wstride * start) + 24;
                const int c = (int)((threadIdx.x & 63u) >> 3);
                pc = c > 0 ? gld(cw + (c - 1)) : 0xFFFFFFFFu;
                pp = gld(cw + 7);
            }
            int tri = walker == 7 ? walk_lone<true>(g, o, d, last, LdsFlat{(CHR_LDS uint32_t *)stacks}, TAIL_STACK * 8,
                                                    LdsFlat{(CHR_LDS uint32_t *)tris}, overflow, sd, it, __builtin_inff(),
                                                    0xFFFFFFFFu, -1, __builtin_inff(), start | WIDE_CHAIN_MORE, true, pc, pp)
                    : walker == 5 ? walk_segment<0, LdsFlat, true>(g, true, o, d, last, 64,
                                                               LdsFlat{(CHR_LDS uint32_t *)stacks}, TAIL_STACK * 8,
                                                               LdsFlat{(CHR_LDS uint32_t *)tris}, top, overflow, sd, it,
                                                               __builtin_inff(), 0xFFFFFFFFu, -1, __builtin_inff(),
                                                               start | WIDE_CHAIN_MORE)
                    : walker >= 3 ? walk_lone<true>(g, o, d, last, LdsFlat{(CHR_LDS uint32_t *)stacks}, TAIL_STACK * 8,
                                                    LdsFlat{(CHR_LDS uint32_t *)tris}, overflow, sd, it, __builtin_inff(),
                                                    0xFFFFFFFFu, -1, __builtin_inff(), start | WIDE_CHAIN_MORE)
                    : pair ? walk_pair(g, top, o, d, last, LdsFlat{(CHR_LDS uint32_t *)stacks}, TAIL_STACK * 8,
                                       (CHR_LDS uint32_t *)tris, 0u, box, walker == 2 ? 2u : PAIR_SPIN_MAX, overflow,
                                       sd, it, lost)
                           : walk_lone(g, o, d, last, LdsFlat{(CHR_LDS uint32_t *)stacks}, TAIL_STACK * 8,
                                       LdsFlat{(CHR_LDS uint32_t *)tris}, overflow, sd, it);
            if (lost)
                tri = walk_lone(g, o, d, last, LdsFlat{(CHR_LDS uint32_t *)stacks}, TAIL_STACK * 8,
                                LdsFlat{(CHR_LDS uint32_t *)tris}, overflow, sd, it);
            const unsigned long long t1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
            if (threadIdx.x == 0) {
                uint32_t *o4 = out + 4 * ((size_t)r * reps + k);
                o4[0] = (uint32_t)tri;
                o4[1] = it;
                o4[2] = (uint32_t)(t1 - t0);
                o4[3] = (uint32_t)(c1 - c0);
            }
        }
    }
    if (walker == 1 || walker == 2) {
        lds_release();
        lds_st(box + PB_STATE, PS_EXIT);
    }
    if (overflow) atomicAdd(out + 4 * (size_t)n * reps, overflow);
}
}  // namespace chr

extern "C" int chr_walk_lone_timing(const chr_geometry *g, const float *d_rays, uint32_t n, uint32_t reps,
                                    uint32_t nwaves, int32_t walker, uint32_t *d_out, void *stream) {
    if (!g || !d_rays || !d_out || nwaves == 0 || reps == 0 || walker < 0 || walker > 7 || walker == 6)
        return chr::fail(CHR_ERR_INVALID, "chr_walk_lone_timing: bad argument");
    if (g->dev.nwnodes == 0) return chr::fail(CHR_ERR_INVALID, "chr_walk_lone_timing: geometry has no wide BVH");
    if (n == 0) return CHR_OK;
    hipLaunchKernelGGL(chr::walk_lone_timing_kernel, dim3(std::min(nwaves, n)), dim3(128), 0, (hipStream_t)stream,
                       (const chr::DevGeom *)g->d_dev, d_rays, n, reps, d_out, walker);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

// The renderer (render.cu, hybrid_render.cu, transform.cu): same translation
// unit, it walks the same BVH and runs the same photon physics.
#include "render.hip"

#ifdef CHR_WALK_PROBE
// ISA inspection only (make probe): walk_segment alone, whole wave, GS = 64 / run-time width
namespace chr {
__global__ __launch_bounds__(BLOCK) void walk_probe_kernel(const DevGeom *__restrict__ gdev, const float *od,
                                                           int *out, int gs) {
    __shared__ uint32_t stacks[(BLOCK / 8) * TAIL_STACK * 2];
    __shared__ uint32_t tris[(BLOCK / 64) * 2 * TAIL_TRI];
    CHR_LDS uint32_t *wstack = (CHR_LDS uint32_t *)stacks + (threadIdx.x >> 6) * 8 * TAIL_STACK * 2;
    CHR_LDS uint32_t *wtris = (CHR_LDS uint32_t *)tris + (threadIdx.x >> 6) * 2 * TAIL_TRI;
    uint32_t overflow = 0, it = 0;
    float sd;
    const V3 o = v3(od[0], od[1], od[2]), d = v3(od[3], od[4], od[5]);
    const TopNodes top{nullptr, 0u};
    const int st = gs == 64 ? walk_segment<64>(*gdev, true, o, d, 7u, 64, LdsFlat{wstack}, TAIL_STACK * 8, LdsFlat{wtris},
                                               top, overflow, sd, it)
                            : walk_segment<0>(*gdev, true, o, d, 7u, gs, LdsFlat{wstack}, TAIL_STACK * gs / 8,
                                              LdsFlat{wtris}, top, overflow, sd, it);
    out[threadIdx.x] = st + (int)overflow + (int)it + (int)sd;
}
}  // namespace chr
#endif
