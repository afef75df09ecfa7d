// wide_bvh.h -- 8-wide quantised BVH used by the gfx950 traversal (see wide_bvh.cpp).
//
// WideNode, 96 bytes = six 16-byte loads:
//   [ 0,16)  origin xyz (f32), biased power-of-two exponent per axis, nchild
//   [16,64)  per-child 8-bit boxes: qlo[x][8] qlo[y][8] qlo[z][8] qhi[x][8] qhi[y][8] qhi[z][8]
//            decoded as fmaf(q, 2^(exp-127), origin) -- always contains the child
//   [64,72)  child_base (first inner child node), tri_base (first triangle record)
//   [72,88)  kind[8]: 0 empty, 1..4 leaf with that many triangles, WIDE_INNER;
//            off[8]:  inner -> node child_base+off, leaf -> records tri_base+off..
// WideTri, 64 bytes = four 16-byte loads (half a 128-byte line): the float32
// vertices v0, v1, v2 (the kernels form the Moller-Trumbore edges v1-v0, v2-v0
// of intersect.h:26-101 and fill_state's normal edge v2-v1, photon.h:365-367,
// with the same float subtractions the reference makes -- so a hit's normal
// comes from the record the walk found and no second triangle array is kept
// in HBM), the original triangle id, its rank in the reference BVH's DFS order
// (the nearest-hit tie-break) and the x/y/z words of its reference leaf node,
// so the kernel applies the reference's own leaf slab test + prune before
// Moller-Trumbore, and the triangle's material code (geometry_types.h: inner,
// outer, surface, the reference's material_codes[id]), so a hit's fill_state
// reads everything it needs from one 64-byte record in four parallel loads.
// The first three loads (v0, v1, v2, id, rank) are the walk's hot part.
#pragma once

#include <cstdint>
#include <vector>

struct chr_geometry_desc;
struct chr_wide_bvh_desc;

namespace chr {

constexpr uint8_t WIDE_INNER = 0x80;

// version of the builder's output (the traversal-BVH cache key, chr_wide_bvh_key):
// bump it whenever the same inputs would build a different tree
constexpr int WIDE_FORMAT = 2;   // 2: no sub-walk cut (round 5)

struct alignas(16) WideNode {
    float origin[3];
    uint8_t exp[3];
    uint8_t nchild;
    uint8_t qlo[3][8];
    uint8_t qhi[3][8];
    uint32_t child_base;
    uint32_t tri_base;
    uint8_t kind[8];
    uint8_t off[8];
    uint32_t pad[2];
};
static_assert(sizeof(WideNode) == 96, "WideNode must be 96 bytes");

struct alignas(16) WideTri {
    float v0[3];
    float v1[3];
    float v2[3];
    uint32_t id;
    uint32_t rank;
    uint32_t leaf[3];      // reference leaf node words x, y, z (lo | hi << 16)
    uint32_t code;         // material code (inner << 24 | outer << 16 | surface << 8)
    uint32_t pad;
};
static_assert(sizeof(WideTri) == 64, "WideTri must be 64 bytes");

struct WideBVH {
    std::vector<WideNode> nodes;   // node 0 is the root
    std::vector<WideTri> tri;      // leaf order
    uint32_t max_depth = 0;        // levels below the root
    uint32_t leaf_max = 0;         // builder setting used
    bool usable = true;            // false: the exact-order traversal must be used
};

// stack capacity of the wide traversal (entries); the builder marks a tree
// whose worst-case stack (7 pushes per level) would not fit as unusable
constexpr int WIDE_STACK = 128;

// Build from the descriptor's mesh and reference BVH (h_nodes).  Returns a chr_status.
int build_wide_bvh(const chr_geometry_desc *d, WideBVH &out);

// The compact form (chr_wide_bvh_desc): record ids / ranks split out of a build.
void wide_compact(const WideBVH &b, std::vector<uint32_t> &rec_id, std::vector<uint32_t> &rec_rank);

// A compact form checked against a geometry, ready to rebuild records from:
// every node / record index in range, the depth within WIDE_STACK, the
// ranks a permutation (rank_rec = its inverse), each record's triangle under a
// reference leaf (leafq: that leaf's x/y/z words per triangle).
struct WideCheck {
    std::vector<uint32_t> rank_rec;
    std::vector<uint32_t> leafq;
    // the tree upward (walk_up): each node's parent as an ancestor word (below;
    // WIDE_NO_PARENT at the root), each record's leaf node
    std::vector<uint32_t> parent;
    std::vector<uint32_t> rec_node;
};
// A device node slot (128 bytes) holds the 96-byte node and, in words 24..31, its
// first 8 ancestors, parent first, as ancestor words: the ancestor's index (bits
// 0-26) | WIDE_CHAIN_MORE (bit 27: set on the 8th when it has ancestors of its own,
// which its slot continues) | the slot of the previous node of the chain in it
// (bits 28-30: the child walk_up skips there) | WIDE_ANCESTOR (bit 31);
// WIDE_NO_PARENT past the root.  A triangle record's last word (pad) is the node
// whose leaf holds it.  walk_up starts a walk at the leaf of the previous hit and
// climbs (node indices < 2^27).
constexpr uint32_t WIDE_NO_PARENT = 0xFFFFFFFFu;
constexpr uint32_t WIDE_NODE_MASK = 0x07FFFFFFu;
constexpr uint32_t WIDE_CHAIN_MORE = 1u << 27;
constexpr uint32_t WIDE_ANCESTOR = 1u << 31;
int wide_validate(const chr_geometry_desc *d, const chr_wide_bvh_desc *w, WideCheck &out);
// the 64-byte triangle records [first, first+n) of a validated compact form
void wide_fill_records(const chr_geometry_desc *d, const chr_wide_bvh_desc *w, const WideCheck &c, size_t first,
                       size_t n, WideTri *out);
// 96-byte nodes [first, first+n) into 128-byte slots (the device layout)
void wide_fill_node_slots(const chr_wide_bvh_desc *w, const WideCheck &c, size_t first, size_t n, uint8_t *out);

}  // namespace chr
