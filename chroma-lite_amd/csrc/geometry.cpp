// geometry.cpp -- chr_geometry_create: upload a flattened, BVH-indexed
// geometry into HBM in the gfx950 traversal layout (device_geometry.h).
// Replaces GPUGeometry.__init__'s device uploads (chroma/gpu/geometry.py:14-526)
// and the Material/Surface/WirePlane make_gpu_struct packing.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/chroma_amd.h"
#include "common.h"
#include "wide_bvh.h"
#include "device_geometry.h"

namespace chr {
std::string &last_error() {
    static thread_local std::string msg;
    return msg;
}
}  // namespace chr

extern "C" const char *chr_last_error(void) { return chr::last_error().c_str(); }

namespace {

struct Blob {
    std::vector<float> data;
    // append n+1 floats (table + its pad element) and return the offset
    uint32_t add(const float *p, uint32_t n_with_pad) {
        uint32_t off = (uint32_t)data.size();
        if (p) data.insert(data.end(), p, p + n_with_pad);
        else data.insert(data.end(), n_with_pad, 0.0f);
        return off;
    }
};

int dev_upload(chr_geometry *g, const void *host, size_t bytes, void **dptr) {
    void *p = nullptr;
    if (bytes == 0) bytes = 16;
    if (g->nallocs >= (int)(sizeof(g->allocs) / sizeof(g->allocs[0])))
        return chr::fail(CHR_ERR_INVALID, "chr_geometry_create: too many device allocations");
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) return chr::fail(CHR_ERR_NOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    g->allocs[g->nallocs++] = p;
    g->bytes += bytes;
    if (host) {
        e = hipMemcpy(p, host, bytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) return chr::fail(CHR_ERR_HIP, "hipMemcpy H2D failed: %s", hipGetErrorString(e));
    }
    *dptr = p;
    return CHR_OK;
}

}  // namespace

extern "C" int chr_geometry_destroy(chr_geometry *g) {
    if (!g) return CHR_OK;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(g->device);
    for (int i = 0; i < g->nallocs; ++i) (void)hipFree(g->allocs[i]);
    (void)hipSetDevice(prev);
    delete g->h_ref_nodes;
    delete g;
    return CHR_OK;
}

// The reference-order walk's data (16-B nodes, 48-B triangles), uploaded on
// first use.  Callers on several host threads may reach it together, and from
// a thread whose current device is not the geometry's: one lock for every
// geometry (first use only), and the allocation on g->device.
int chr::geometry_ref_nodes(const chr_geometry *cg) {
    static std::mutex m;
    std::lock_guard<std::mutex> lock(m);
    chr_geometry *g = const_cast<chr_geometry *>(cg);
    if (!g->h_ref_nodes && !g->ref_tri_pending) return CHR_OK;
    int prev = 0;
    hipError_t e = hipGetDevice(&prev);
    if (e == hipSuccess && prev != g->device) e = hipSetDevice(g->device);
    if (e != hipSuccess) return chr::fail(CHR_ERR_HIP, "geometry_ref_nodes: device %d: %s", g->device, hipGetErrorString(e));
    auto run = [&]() -> int {
        void *p = nullptr;
        int rc;
        if (g->h_ref_nodes) {
            if ((rc = dev_upload(g, g->h_ref_nodes->data(), g->h_ref_nodes->size() * sizeof(uint4), &p))) return rc;
            g->dev.nodes = (const uint4 *)p;
            delete g->h_ref_nodes;
            g->h_ref_nodes = nullptr;
        }
        if (g->ref_tri_pending) {
            if ((rc = dev_upload(g, nullptr, (size_t)g->dev.ntriangles * 48, &p))) return rc;
            if ((rc = chr::build_ref_triangles(g->dev, (float4 *)p))) return rc;
            g->dev.tri = (const float4 *)p;
            g->ref_tri_pending = false;
        }
        const hipError_t e2 = hipMemcpy(g->d_dev, &g->dev, sizeof(g->dev), hipMemcpyHostToDevice);
        if (e2 != hipSuccess) return chr::fail(CHR_ERR_HIP, "hipMemcpy H2D failed: %s", hipGetErrorString(e2));
        return CHR_OK;
    };
    const int rc = run();
    if (prev != g->device) (void)hipSetDevice(prev);
    return rc;
}

extern "C" int chr_geometry_device_bytes(const chr_geometry *g, uint64_t *bytes) {
    if (!g || !bytes) return chr::fail(CHR_ERR_INVALID, "chr_geometry_device_bytes: null argument");
    *bytes = g->bytes;
    return CHR_OK;
}

extern "C" int chr_geometry_create(const chr_geometry_desc *d, chr_geometry **out) {
    if (!d || !out) return chr::fail(CHR_ERR_INVALID, "chr_geometry_create: null argument");
    if (d->ntriangles == 0 || d->nnodes == 0 || !d->h_vertices || !d->h_triangles || !d->h_nodes ||
        !d->h_material_codes)
        return chr::fail(CHR_ERR_INVALID, "chr_geometry_create: empty mesh or BVH");
    if (d->nmaterials == 0 || !d->materials) return chr::fail(CHR_ERR_INVALID, "chr_geometry_create: no materials");
    if (d->nwireplanes && !d->wireplanes) return chr::fail(CHR_ERR_INVALID, "chr_geometry_create: wireplanes NULL");
    if (d->wavelength_n < 2 || d->time_n < 2) return chr::fail(CHR_ERR_INVALID, "chr_geometry_create: grids need >= 2 points");
    // validate triangle indices / BVH child ranges up front: an out-of-range
    // index would otherwise become an out-of-bounds read inside the kernel.
    for (size_t i = 0; i < (size_t)d->ntriangles * 3; ++i)
        if (d->h_triangles[i] >= d->nvertices)
            return chr::fail(CHR_ERR_INVALID, "triangle %zu references vertex %u >= %u", i / 3, d->h_triangles[i], d->nvertices);
    for (size_t i = 0; i < d->nnodes; ++i) {
        const uint32_t w = d->h_nodes[4 * i + 3];
        const uint32_t nc = w >> 28, child = w & 0x0FFFFFFFu;
        if (nc == 0 ? child >= d->ntriangles : (uint64_t)child + nc > d->nnodes)
            return chr::fail(CHR_ERR_INVALID, "BVH node %zu has child %u nchild %u out of range", i, child, nc);
    }
    for (size_t t = 0; t < d->ntriangles; ++t) {
        const uint32_t c = d->h_material_codes[t];
        int m1 = (c >> 24) & 0xFF, m2 = (c >> 16) & 0xFF, s = (c >> 8) & 0xFF;
        if (m1 >= (int)d->nmaterials || m2 >= (int)d->nmaterials)
            return chr::fail(CHR_ERR_INVALID, "triangle %zu: material index out of range", t);
        if (s != 0xFF && (s >= (int)d->nsurfaces || !d->surfaces || !d->surfaces[s].present))
            return chr::fail(CHR_ERR_INVALID, "triangle %zu: surface %d missing", t, s);
    }

    chr_geometry *g = new (std::nothrow) chr_geometry();
    if (!g) return chr::fail(CHR_ERR_NOMEM, "chr_geometry_create: host allocation failed");
    std::memset(g, 0, sizeof(*g));
    (void)hipGetDevice(&g->device);
    int rc = CHR_OK;
    try {
        chr::DevGeom &dg = g->dev;
        dg.ox = d->world_origin[0]; dg.oy = d->world_origin[1]; dg.oz = d->world_origin[2];
        dg.scale = d->world_scale;
        dg.nnodes = d->nnodes; dg.ntriangles = d->ntriangles; dg.nwireplanes = d->nwireplanes;
        dg.wl_n = d->wavelength_n; dg.wl_start = d->wavelength_start; dg.wl_step = d->wavelength_step;
        dg.t_n = d->time_n; dg.t_start = d->time_start; dg.t_step = d->time_step;

        void *p;
        {
            chr::WideBVH wb;
            if ((rc = chr::build_wide_bvh(d, wb))) throw rc;
            if (wb.usable && !std::getenv("CHR_EXACT_ORDER_ONLY")) {
                // nodes padded to 128 bytes: one node = one cache line (a 96-byte node at a
                // 96-byte stride straddles two lines half the time).  r01: no gain over the
                // packed stride; r03 ab21, where the later steps' walks are line-bound:
                // 463.7 -> 467.1 M/s, so the padded slots are the default (the packed ones
                // kept beside them with CHR_NODE_LAYOUT_AB, selected by CHR_NODE_LAYOUT=96)
                const bool ab = std::getenv("CHR_NODE_LAYOUT_AB") != nullptr;
                std::vector<uint8_t> padded(wb.nodes.size() * 128, 0);
                for (size_t i = 0; i < wb.nodes.size(); ++i)
                    std::memcpy(padded.data() + 128 * i, &wb.nodes[i], sizeof(chr::WideNode));
                if ((rc = dev_upload(g, padded.data(), std::max<size_t>(128, padded.size()), &p))) throw rc;
                dg.wnodes = (const uint4 *)p;
                dg.wstride = 8;
                std::vector<uint8_t>().swap(padded);
                if (ab) {
                    if ((rc = dev_upload(g, wb.nodes.data(), wb.nodes.size() * sizeof(chr::WideNode), &p))) throw rc;
                    g->wnodes_alt = (const uint4 *)p;
                    g->wstride_alt = 6;
                }
                if ((rc = dev_upload(g, wb.tri.data(), std::max<size_t>(1, wb.tri.size()) * sizeof(chr::WideTri), &p)))
                    throw rc;
                dg.wtri = (const float4 *)p;
                dg.nwnodes = (uint32_t)wb.nodes.size();
                dg.nwtri = (uint32_t)wb.tri.size();
                if ((rc = dev_upload(g, wb.cut.data(), wb.cut.size() * 4, &p))) throw rc;
                dg.wcut = (const uint2 *)p;
                dg.nwcut = (uint32_t)(wb.cut.size() / 2);
                if ((rc = dev_upload(g, wb.rank_rec.data(), wb.rank_rec.size() * 4, &p))) throw rc;
                dg.wrank_rec = (const uint32_t *)p;
            }
        }

        // de-indexed reference triangle records (v0, e1 = v1-v0, e2 = v2-v0,
        // e3 = v2-v1) for the reference walk: uploaded now only without a wide
        // BVH (or with CHR_REF_NODES_RESIDENT); otherwise built on the device
        // from the wide records the first time a call walks the reference BVH
        if (dg.nwnodes == 0 || std::getenv("CHR_REF_NODES_RESIDENT")) {
            std::vector<float> tri((size_t)d->ntriangles * 12);
            const float *v = d->h_vertices;
#pragma omp parallel for schedule(static)
            for (int64_t t = 0; t < (int64_t)d->ntriangles; ++t) {
                const uint32_t *ix = d->h_triangles + 3 * t;
                const float *a = v + 3 * (size_t)ix[0], *b = v + 3 * (size_t)ix[1], *c = v + 3 * (size_t)ix[2];
                float *r = tri.data() + 12 * t;
                r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
                r[3] = b[0] - a[0]; r[4] = b[1] - a[1]; r[5] = b[2] - a[2];
                r[6] = c[0] - a[0]; r[7] = c[1] - a[1]; r[8] = c[2] - a[2];
                r[9] = c[0] - b[0]; r[10] = c[1] - b[1]; r[11] = c[2] - b[2];
            }
            if ((rc = dev_upload(g, tri.data(), tri.size() * sizeof(float), &p))) throw rc;
            dg.tri = (const float4 *)p;
        } else {
            g->ref_tri_pending = true;
        }

        // reference BVH nodes: all resident only without a wide BVH (or with
        // CHR_REF_NODES_RESIDENT); otherwise the root, the rest on first use
        if (dg.nwnodes == 0 || std::getenv("CHR_REF_NODES_RESIDENT")) {
            if ((rc = dev_upload(g, d->h_nodes, (size_t)d->nnodes * 16, &p))) throw rc;
        } else {
            g->h_ref_nodes = new std::vector<uint4>((const uint4 *)d->h_nodes, (const uint4 *)d->h_nodes + d->nnodes);
            if ((rc = dev_upload(g, d->h_nodes, 16, &p))) throw rc;
        }
        dg.nodes = (const uint4 *)p;

        if ((rc = dev_upload(g, d->h_material_codes, (size_t)d->ntriangles * 4, &p))) throw rc;
        dg.material_codes = (const uint32_t *)p;

        Blob blob, comp;
        const uint32_t W1 = d->wavelength_n + 1, T1 = d->time_n + 1;
        std::vector<chr::DevMaterial> mats(d->nmaterials);
        for (uint32_t i = 0; i < d->nmaterials; ++i) {
            const chr_material_desc &m = d->materials[i];
            chr::DevMaterial &o = mats[i];
            if (!m.refractive_index || !m.absorption_length || !m.scattering_length) {
                rc = chr::fail(CHR_ERR_INVALID, "material %u: missing table", i);
                throw rc;
            }
            o.num_comp = m.num_comp;
            o.refractive_index = blob.add(m.refractive_index, W1);
            o.absorption_length = blob.add(m.absorption_length, W1);
            o.scattering_length = blob.add(m.scattering_length, W1);
            // the components' tables (bulk re-emission, 20,000-entry time CDFs) go in a
            // second blob after the records: the hot part before them fits in LDS
            o.comp_reemission_prob = (uint32_t)comp.data.size();
            for (uint32_t c = 0; c < m.num_comp; ++c) comp.add(m.comp_reemission_prob + c * W1, W1);
            o.comp_reemission_wvl_cdf = (uint32_t)comp.data.size();
            for (uint32_t c = 0; c < m.num_comp; ++c) comp.add(m.comp_reemission_wvl_cdf + c * W1, W1);
            o.comp_reemission_time_cdf = (uint32_t)comp.data.size();
            for (uint32_t c = 0; c < m.num_comp; ++c) comp.add(m.comp_reemission_time_cdf + c * T1, T1);
            o.comp_absorption_length = (uint32_t)comp.data.size();
            for (uint32_t c = 0; c < m.num_comp; ++c) comp.add(m.comp_absorption_length + c * W1, W1);
        }
        std::vector<chr::DevSurface> surfs(d->nsurfaces > 0 ? d->nsurfaces : 1);
        std::memset(surfs.data(), 0, surfs.size() * sizeof(chr::DevSurface));
        for (uint32_t i = 0; i < d->nsurfaces; ++i) {
            const chr_surface_desc &s = d->surfaces[i];
            chr::DevSurface &o = surfs[i];
            o.present = s.present ? 1u : 0u;
            if (!s.present) continue;
            o.model = s.model; o.transmissive = s.transmissive; o.thickness = s.thickness;
            o.detect = blob.add(s.detect, W1);
            o.absorb = blob.add(s.absorb, W1);
            o.reemit = blob.add(s.reemit, W1);
            o.reflect_diffuse = blob.add(s.reflect_diffuse, W1);
            o.reflect_specular = blob.add(s.reflect_specular, W1);
            o.eta = blob.add(s.eta, W1);
            o.k = blob.add(s.k, W1);
            o.reemission_cdf = blob.add(s.reemission_cdf, W1);
            if (s.model == CHR_SURFACE_DICHROIC && s.dichroic_nangles == 0) {
                rc = chr::fail(CHR_ERR_INVALID, "surface %u: dichroic model without DichroicProps", i);
                throw rc;
            }
            if (s.model == CHR_SURFACE_ANGULAR && s.angular_nangles == 0) {
                rc = chr::fail(CHR_ERR_INVALID, "surface %u: angular model without AngularProps", i);
                throw rc;
            }
            o.dichroic_nangles = s.dichroic_nangles;
            if (s.dichroic_nangles) {
                o.dichroic_angles = blob.add(s.dichroic_angles, s.dichroic_nangles);
                o.dichroic_reflect = (uint32_t)blob.data.size();
                blob.data.insert(blob.data.end(), s.dichroic_reflect, s.dichroic_reflect + (size_t)s.dichroic_nangles * W1);
                o.dichroic_transmit = (uint32_t)blob.data.size();
                blob.data.insert(blob.data.end(), s.dichroic_transmit, s.dichroic_transmit + (size_t)s.dichroic_nangles * W1);
            }
            o.angular_nangles = s.angular_nangles;
            if (s.angular_nangles) {
                o.angular_angles = blob.add(s.angular_angles, s.angular_nangles);
                o.angular_transmit = blob.add(s.angular_transmit, s.angular_nangles);
                o.angular_reflect_specular = blob.add(s.angular_reflect_specular, s.angular_nangles);
                o.angular_reflect_diffuse = blob.add(s.angular_reflect_diffuse, s.angular_nangles);
            }
        }
        {   // one allocation [tables | materials | surfaces], 16-byte aligned parts (DevGeom::phys)
            std::vector<uint32_t> phys(blob.data.size());
            std::memcpy(phys.data(), blob.data.data(), blob.data.size() * 4);
            phys.resize((phys.size() + 3) & ~(size_t)3, 0u);
            const uint32_t mat_off = (uint32_t)phys.size();
            phys.resize(phys.size() + mats.size() * sizeof(chr::DevMaterial) / 4);
            std::memcpy(phys.data() + mat_off, mats.data(), mats.size() * sizeof(chr::DevMaterial));
            phys.resize((phys.size() + 3) & ~(size_t)3, 0u);
            const uint32_t surf_off = (uint32_t)phys.size();
            phys.resize(phys.size() + surfs.size() * sizeof(chr::DevSurface) / 4);
            std::memcpy(phys.data() + surf_off, surfs.data(), surfs.size() * sizeof(chr::DevSurface));
            phys.resize((phys.size() + 3) & ~(size_t)3, 0u);
            const uint32_t hot = (uint32_t)phys.size();
            // material component offsets: relative to the phys base, past the records
            for (auto &m : mats) {
                m.comp_reemission_prob += hot;
                m.comp_reemission_wvl_cdf += hot;
                m.comp_reemission_time_cdf += hot;
                m.comp_absorption_length += hot;
            }
            std::memcpy(phys.data() + mat_off, mats.data(), mats.size() * sizeof(chr::DevMaterial));
            phys.resize(phys.size() + comp.data.size());
            std::memcpy(phys.data() + hot, comp.data.data(), comp.data.size() * 4);
            phys.resize((phys.size() + 3) & ~(size_t)3, 0u);
            if ((rc = dev_upload(g, phys.data(), phys.size() * 4, &p))) throw rc;
            dg.phys = (const uint32_t *)p;
            dg.phys_words = (uint32_t)phys.size();
            dg.phys_hot_words = hot;
            dg.mat_off = mat_off;
            dg.surf_off = surf_off;
            dg.tables = (const float *)p;
            dg.tables_g = (const float *)p;
            dg.materials = (const chr::DevMaterial *)(dg.phys + mat_off);
            dg.surfaces = (const chr::DevSurface *)(dg.phys + surf_off);
        }
        if (d->nwireplanes) {
            if ((rc = dev_upload(g, d->wireplanes, (size_t)d->nwireplanes * sizeof(chr_wireplane_desc), &p))) throw rc;
            dg.wireplanes = (const chr_wireplane_desc *)p;
        }
        if ((rc = dev_upload(g, &dg, sizeof(dg), &p))) throw rc;
        g->d_dev = p;
    } catch (int code) {
        chr_geometry_destroy(g);
        return code;
    } catch (const std::bad_alloc &) {
        chr_geometry_destroy(g);
        return chr::fail(CHR_ERR_NOMEM, "chr_geometry_create: host allocation failed");
    }
    *out = g;
    return CHR_OK;
}
