// device_geometry.h -- HBM layout of a geometry on gfx950.
//
// Reference layout (chroma/cuda/geometry_types.h:124-139, gpu/geometry.py:389-520):
// a Geometry struct of pointers, copied into __shared__ by every block,
// double pointer chase (materials[i]->refractive_index[j]) per table lookup,
// triangles as index triples into a vertex array (4 dependent loads/triangle).
//
// Here:
//  * DevGeom lives in device memory and kernels take a `const DevGeom *__restrict__`:
//    its fields are uniform scalar loads, and passing it to out-of-line helpers
//    passes a pointer (a by-value kernel argument whose address escapes gets
//    copied into every work-item's scratch);
//  * BVH nodes stay the reference's 16-byte quantised uint4 (the exact-order
//    traversal variant walks them; resident in HBM only once a call needs them,
//    chr::geometry_ref_nodes); the default traversal walks an 8-wide SAH
//    BVH built over the same leaf boxes with the reference DFS rank as the
//    nearest-hit tie-break (wide_bvh.h) -- same answers, far fewer nodes;
//  * the wide BVH's 64-byte triangle records (v0, v1, v2, id, rank, leaf box;
//    wide_bvh.h) serve the walk AND the hit's normal; the reference walk's
//    de-indexed 48-byte records of three float4
//        (v0.x v0.y v0.z e1.x) (e1.y e1.z e2.x e2.y) (e2.z e3.x e3.y e3.z)
//    with e1 = v1-v0, e2 = v2-v0 (the Moller-Trumbore edges, intersect.h:26-101)
//    and e3 = v2-v1 (the normal edge of fill_state, photon.h:365-367) are
//    resident only once a call walks the reference BVH (built on the device
//    from the wide records, chr::geometry_ref_nodes);
//  * every wavelength / time table lives in one float blob (each table padded
//    by one element, see chr_geometry_desc), addressed by 32-bit offsets held
//    in small DevMaterial / DevSurface records.
#pragma once
#include <vector>

#include <cstdint>

#include "../../include/chroma_amd.h"

namespace chr {

// buckets of a re-emission time CDF's index (geometry.cpp time_cdf_index)
constexpr uint32_t TIME_INDEX_BUCKETS = 4096;

struct DevMaterial {
    uint32_t num_comp;
    uint32_t refractive_index, absorption_length, scattering_length;       // blob offsets
    // first component; component c at + c * (wl_n + 1) (time CDF: + c * (t_n + 1))
    uint32_t comp_reemission_prob, comp_reemission_wvl_cdf, comp_absorption_length;   // hot
    uint32_t comp_reemission_time_cdf;                                     // cold (tables_g)
    uint32_t comp_time_index;   // cold: (TIME_INDEX_BUCKETS + 1) words per component, ~0u: none
};

struct DevSurface {
    uint32_t present, model, transmissive;
    float thickness;
    uint32_t detect, absorb, reemit, reflect_diffuse, reflect_specular, eta, k, reemission_cdf;
    uint32_t dichroic_nangles, dichroic_angles, dichroic_reflect, dichroic_transmit;
    uint32_t angular_nangles, angular_angles, angular_transmit, angular_reflect_specular,
        angular_reflect_diffuse;
};

struct DevGeom {
    const uint4 *nodes;
    const float4 *tri;               // 3 float4 per triangle (reference walk; resident on first use)
    const uint32_t *material_codes;
    const float *tables;
    const DevMaterial *materials;
    const DevSurface *surfaces;
    const chr_wireplane_desc *wireplanes;
    const uint4 *wnodes;             // 8-wide SAH BVH, node i at wnodes[wstride * i] (wide_bvh.h)
    const float4 *wtri;              // 3 float4 per leaf triangle record (wide_bvh.h)
    uint32_t nwnodes, nwtri;
    uint32_t wstride;                // uint4 per node slot: 8 (each 96-byte node padded to one 128-byte line)
    float ox, oy, oz, scale;         // world_origin, world_scale
    uint32_t nnodes, ntriangles, nwireplanes;
    uint32_t wl_n;
    float wl_start, wl_step;
    uint32_t t_n;
    float t_start, t_step;
    // the physics tables as one allocation, [tables | materials | surfaces]: tables ==
    // phys, materials == phys + mat_off, surfaces == phys + surf_off (words), phys_words
    // in all -- small enough on the usual detectors (demo: 25 KB) for the shade and
    // tail kernels to keep a copy in LDS (chr::PhysCache)
    const uint32_t *phys;
    uint32_t phys_words, mat_off, surf_off;
    // [0, phys_hot_words): the tables (identical ones stored once) and records; after it
    // the materials' re-emission time CDFs and their bucket indexes, read through tables_g
    // (== tables in global memory; phys_cache points tables into LDS, tables_g stays)
    uint32_t phys_hot_words;
    const float *tables_g;
};

}  // namespace chr

struct chr_geometry {
    chr::DevGeom dev;
    void *d_dev;          // a device copy of dev: kernels take `const DevGeom *` (uniform scalar loads)
    int device;
    uint64_t bytes;
    void *allocs[16];
    int nallocs;
    // The reference BVH nodes (16 B each) are walked only by the exact-order
    // variant, the no-wide-BVH fallback and distance_to_mesh's exact form.  With a
    // wide BVH only the root stays in HBM (the renderer's world box) and the
    // rest waits here until chr_geometry_ref_nodes() uploads it (once).
    std::vector<uint4> *h_ref_nodes;
    bool ref_tri_pending;   // the 48-byte reference triangle records are built on first use
};
namespace chr {
// the bucket index of ncomp CDFs of n entries (CDF c at cdf0 + c * stride):
// (TIME_INDEX_BUCKETS + 1) words per CDF (sample_cdf_indexed, sampling.h); false
// when one is not >= 2 finite non-decreasing entries (no index: plain bisection)
bool time_cdf_index(const float *cdf0, uint32_t ncomp, uint32_t n, uint32_t stride, std::vector<uint32_t> &idx);
// make every reference node and the reference triangle records resident in
// HBM (no-op when they are); CHR_OK or an error
int geometry_ref_nodes(const chr_geometry *g);
// fill the 48-byte reference triangle records from the wide records (propagate.hip)
int build_ref_triangles(const DevGeom &dg, float4 *tri);
}
