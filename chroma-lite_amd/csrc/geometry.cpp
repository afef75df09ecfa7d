// geometry.cpp -- chr_geometry_create: upload a flattened, BVH-indexed
// geometry into HBM in the gfx950 traversal layout (device_geometry.h).
// Replaces GPUGeometry.__init__'s device uploads (chroma/gpu/geometry.py:14-526)
// and the Material/Surface/WirePlane make_gpu_struct packing.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <unordered_map>
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

// Physics tables as 32-bit words.  add() appends a block (a table with its pad
// element, or a group of tables addressed from one offset) and returns its
// offset; a block identical to one already added shares that copy (detectors
// repeat the same tables across materials and surfaces, and the hot part has
// to fit LDS, PhysCache in propagate.hip).
struct Blob {
    std::vector<uint32_t> data;
    std::unordered_map<std::string, uint32_t> seen;
    uint32_t add(const void *p, size_t nwords) {
        if (nwords == 0) return (uint32_t)data.size();
        std::string key(nwords * 4, '\0');
        if (p) std::memcpy(&key[0], p, nwords * 4);
        auto it = seen.find(key);
        if (it != seen.end()) return it->second;
        const uint32_t off = (uint32_t)data.size();
        data.resize(data.size() + nwords);
        std::memcpy(data.data() + off, key.data(), nwords * 4);
        seen.emplace(std::move(key), off);
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

// The bucket index of a re-emission time CDF (sample_cdf_indexed, sampling.h):
// per component TIME_INDEX_BUCKETS+1 words, word b = the largest j with
// cdf[j] <= b/TIME_INDEX_BUCKETS clamped to [0, n-2].  Only for CDFs of >= 2
// finite non-decreasing entries (false otherwise: the kernel bisects the whole
// table as the reference does, random.h:34-55).
bool chr::time_cdf_index(const float *cdf0, uint32_t ncomp, uint32_t n, uint32_t stride, std::vector<uint32_t> &idx) {
    if (n < 2 || ncomp == 0) return false;
    for (uint32_t c = 0; c < ncomp; ++c) {
        const float *cdf = cdf0 + (size_t)c * stride;
        for (uint32_t j = 0; j < n; ++j)
            if (!std::isfinite(cdf[j]) || (j + 1 < n && !(cdf[j] <= cdf[j + 1]))) return false;
    }
    const uint32_t NB = chr::TIME_INDEX_BUCKETS;
    idx.assign((size_t)ncomp * (NB + 1), 0u);
    for (uint32_t c = 0; c < ncomp; ++c) {
        const float *cdf = cdf0 + (size_t)c * stride;
        for (uint32_t b = 0; b <= NB; ++b) {
            const float x = (float)b / (float)NB;          // exact: NB is a power of two
            const int64_t cnt = std::upper_bound(cdf, cdf + n, x) - cdf;
            idx[(size_t)c * (NB + 1) + b] = (uint32_t)std::min<int64_t>(std::max<int64_t>(cnt - 1, 0), n - 2);
        }
    }
    return true;
}

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

extern "C" int chr_geometry_phys_words(const chr_geometry *g, uint32_t *hot_words, uint32_t *total_words) {
    if (!g || !hot_words || !total_words) return chr::fail(CHR_ERR_INVALID, "chr_geometry_phys_words: null argument");
    *hot_words = g->dev.phys_hot_words;
    *total_words = g->dev.phys_words;
    return CHR_OK;
}

// Host staging for the large uploads: records / node slots are filled chunk by
// chunk into two pinned buffers while the previous chunk's copy runs, so the
// 64-byte records (10.9 GB on the 29k detector) never exist whole in host memory.
// Without pinned memory the chunks go through one pageable buffer, synchronously.
struct Stager {
    static constexpr size_t CHUNK = 64u << 20;
    hipStream_t stream = nullptr;
    void *buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
    std::vector<uint8_t> pageable;
    int init() {
        if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) stream = nullptr;
        for (int k = 0; k < 2 && stream; ++k) {
            if (hipHostMalloc(&buf[k], CHUNK, hipHostMallocDefault) != hipSuccess ||
                hipEventCreateWithFlags(&ev[k], hipEventDisableTiming) != hipSuccess) {
                release();
                break;
            }
        }
        if (!buf[0]) pageable.resize(CHUNK);
        return CHR_OK;
    }
    void release() {
        if (stream) (void)hipStreamSynchronize(stream);
        for (int k = 0; k < 2; ++k) {
            if (buf[k]) (void)hipHostFree(buf[k]);
            if (ev[k]) (void)hipEventDestroy(ev[k]);
            buf[k] = nullptr;
            ev[k] = nullptr;
        }
        if (stream) (void)hipStreamDestroy(stream);
        stream = nullptr;
    }
    ~Stager() { release(); }
    // buffer k (0/1) once its previous copy has finished
    int acquire(int k, uint8_t **p) {
        if (!buf[0]) { *p = pageable.data(); return CHR_OK; }
        if (used[k]) CHR_HIP_CHECK(hipEventSynchronize(ev[k]));
        *p = static_cast<uint8_t *>(buf[k]);
        return CHR_OK;
    }
    int copy(int k, void *dst, size_t bytes) {
        if (!buf[0]) {
            CHR_HIP_CHECK(hipMemcpy(dst, pageable.data(), bytes, hipMemcpyHostToDevice));
            return CHR_OK;
        }
        CHR_HIP_CHECK(hipMemcpyAsync(dst, buf[k], bytes, hipMemcpyHostToDevice, stream));
        CHR_HIP_CHECK(hipEventRecord(ev[k], stream));
        used[k] = true;
        return CHR_OK;
    }
    int finish() {
        if (stream) CHR_HIP_CHECK(hipStreamSynchronize(stream));
        return CHR_OK;
    }
};

// the traversal BVH (compact form w) into HBM: 96-byte nodes in 128-byte slots
// (one line per node: r01 no gain over the packed stride; r03 ab21, where the
// later steps' walks are line-bound, 463.7 -> 467.1 M/s), the 64-byte triangle
// records rebuilt from the geometry
static int upload_wide(chr_geometry *g, const chr_geometry_desc *d, const chr_wide_bvh_desc *w) {
    chr::WideCheck c;
    CHR_TRY(chr::wide_validate(d, w, c));
    chr::DevGeom &dg = g->dev;
    Stager st;
    CHR_TRY(st.init());
    void *p = nullptr;
    int k = 0;
    CHR_TRY(dev_upload(g, nullptr, std::max<size_t>(128, (size_t)w->nnodes * 128), &p));
    dg.wnodes = (const uint4 *)p;
    dg.wstride = 8;
    for (size_t i = 0, per = Stager::CHUNK / 128; i < w->nnodes; i += per, k ^= 1) {
        const size_t n = std::min<size_t>(per, w->nnodes - i);
        uint8_t *h;
        CHR_TRY(st.acquire(k, &h));
        chr::wide_fill_node_slots(w, c, i, n, h);
        CHR_TRY(st.copy(k, static_cast<uint8_t *>(p) + 128 * i, n * 128));
    }
    CHR_TRY(dev_upload(g, nullptr, std::max<size_t>(1, w->nrec) * sizeof(chr::WideTri), &p));
    dg.wtri = (const float4 *)p;
    for (size_t i = 0, per = Stager::CHUNK / sizeof(chr::WideTri); i < w->nrec; i += per, k ^= 1) {
        const size_t n = std::min<size_t>(per, w->nrec - i);
        uint8_t *h;
        CHR_TRY(st.acquire(k, &h));
        chr::wide_fill_records(d, w, c, i, n, reinterpret_cast<chr::WideTri *>(h));
        CHR_TRY(st.copy(k, static_cast<uint8_t *>(p) + sizeof(chr::WideTri) * i, n * sizeof(chr::WideTri)));
    }
    CHR_TRY(st.finish());
    dg.nwnodes = w->nnodes;
    dg.nwtri = w->nrec;
    return CHR_OK;
}

// create with the traversal BVH given in compact form (w, validated first), or
// built here (w == NULL)
static int geometry_create(const chr_geometry_desc *d, const chr_wide_bvh_desc *w, chr_geometry **out) {
    if (!d || !out) return chr::fail(CHR_ERR_INVALID, "chr_geometry_create: null argument");
    if (d->ntriangles == 0 || d->nnodes == 0 || !d->h_vertices || !d->h_triangles || !d->h_nodes ||
        !d->h_material_codes)
        return chr::fail(CHR_ERR_INVALID, "chr_geometry_create: empty mesh or BVH");
    if (d->nmaterials == 0 || !d->materials) return chr::fail(CHR_ERR_INVALID, "chr_geometry_create: no materials");
    if (d->nwireplanes && !d->wireplanes) return chr::fail(CHR_ERR_INVALID, "chr_geometry_create: wireplanes NULL");
    if (d->wavelength_n < 2 || d->time_n < 2) return chr::fail(CHR_ERR_INVALID, "chr_geometry_create: grids need >= 2 points");
    // validate triangle indices / BVH child ranges / material codes up front: an
    // out-of-range index would otherwise become an out-of-bounds read inside the kernel
    int64_t bad_tri = -1, bad_node = -1, bad_code = -1;
    const int64_t NT = d->ntriangles, NN = d->nnodes;
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static) reduction(max : bad_tri, bad_code)
    for (int64_t t = 0; t < NT; ++t) {
        const uint32_t *ix = d->h_triangles + 3 * t;
        if (ix[0] >= d->nvertices || ix[1] >= d->nvertices || ix[2] >= d->nvertices) bad_tri = std::max(bad_tri, t);
        const uint32_t c = d->h_material_codes[t];
        const uint32_t m1 = (c >> 24) & 0xFF, m2 = (c >> 16) & 0xFF, sf = (c >> 8) & 0xFF;
        if (m1 >= d->nmaterials || m2 >= d->nmaterials ||
            (sf != 0xFF && (sf >= d->nsurfaces || !d->surfaces || !d->surfaces[sf].present)))
            bad_code = std::max(bad_code, t);
    }
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static) reduction(max : bad_node)
    for (int64_t i = 0; i < NN; ++i) {
        const uint32_t w = d->h_nodes[4 * i + 3];
        const uint32_t nc = w >> 28, child = w & 0x0FFFFFFFu;
        if (nc == 0 ? child >= d->ntriangles : (uint64_t)child + nc > d->nnodes) bad_node = std::max(bad_node, i);
    }
    if (bad_tri >= 0)
        return chr::fail(CHR_ERR_INVALID, "triangle %lld references a vertex >= %u", (long long)bad_tri, d->nvertices);
    if (bad_node >= 0)
        return chr::fail(CHR_ERR_INVALID, "BVH node %lld has a child out of range", (long long)bad_node);
    if (bad_code >= 0)
        return chr::fail(CHR_ERR_INVALID, "triangle %lld: material index out of range or surface missing", (long long)bad_code);

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
            // the traversal BVH in compact form: given (a cache), or built now and
            // compacted, so both paths upload through the same record fill
            chr::WideBVH wb;
            std::vector<uint32_t> rec_id, rec_rank;
            chr_wide_bvh_desc built;
            std::memset(&built, 0, sizeof(built));
            const bool exact_only = std::getenv("CHR_EXACT_ORDER_ONLY") != nullptr;
            if (w && (!w->usable || exact_only)) {
                w = nullptr;       // a tree the wide walk cannot use: the exact-order walk, nothing built
            } else if (!w) {
                if ((rc = chr::build_wide_bvh(d, wb))) throw rc;
                chr::wide_compact(wb, rec_id, rec_rank);
                std::vector<chr::WideTri>().swap(wb.tri);
                built.nnodes = (uint32_t)wb.nodes.size();
                built.nrec = (uint32_t)rec_id.size();
                built.max_depth = wb.max_depth;
                built.usable = wb.usable ? 1 : 0;
                built.leaf_max = wb.leaf_max;
                built.h_nodes = wb.nodes.data();
                built.h_rec_id = rec_id.data();
                built.h_rec_rank = rec_rank.data();
                if (built.usable && !exact_only) w = &built;
            }
            if (w) {
                if ((rc = upload_wide(g, d, w))) throw rc;
            }
        }

        // de-indexed reference triangle records (v0, e1 = v1-v0, e2 = v2-v0,
        // e3 = v2-v1) for the reference walk: uploaded now only without a wide
        // BVH; otherwise built on the device from the wide records the first
        // time a call walks the reference BVH
        if (dg.nwnodes == 0) {
            std::vector<float> tri((size_t)d->ntriangles * 12);
            const float *v = d->h_vertices;
#pragma omp parallel for num_threads(chr::host_threads()) schedule(static)
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

        // reference BVH nodes: all resident only without a wide BVH; otherwise
        // the root, the rest on first use
        if (dg.nwnodes == 0) {
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
            // the components' wavelength tables (a group each, component c at + c*W1) stay
            // with the hot tables; the 20,000-entry time CDFs and their bucket index go in a
            // second blob after the records (read from HBM: the hot part fits LDS)
            const size_t nc = m.num_comp;
            o.comp_reemission_prob = blob.add(m.comp_reemission_prob, nc * W1);
            o.comp_reemission_wvl_cdf = blob.add(m.comp_reemission_wvl_cdf, nc * W1);
            o.comp_absorption_length = blob.add(m.comp_absorption_length, nc * W1);
            o.comp_reemission_time_cdf = comp.add(m.comp_reemission_time_cdf, nc * T1);
            o.comp_time_index = ~0u;
            std::vector<uint32_t> idx;
            if (nc && chr::time_cdf_index(m.comp_reemission_time_cdf, m.num_comp, d->time_n, T1, idx))
                o.comp_time_index = comp.add(idx.data(), idx.size());
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
                o.dichroic_reflect = blob.add(s.dichroic_reflect, (size_t)s.dichroic_nangles * W1);
                o.dichroic_transmit = blob.add(s.dichroic_transmit, (size_t)s.dichroic_nangles * W1);
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
            std::vector<uint32_t> phys(blob.data);
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
            // the cold offsets: relative to the phys base, past the records
            for (auto &m : mats) {
                m.comp_reemission_time_cdf += hot;
                if (m.comp_time_index != ~0u) m.comp_time_index += hot;
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

extern "C" int chr_geometry_create(const chr_geometry_desc *d, chr_geometry **out) {
    return geometry_create(d, nullptr, out);
}

extern "C" int chr_geometry_create_wide(const chr_geometry_desc *d, const chr_wide_bvh_desc *w, chr_geometry **out) {
    if (!w) return chr::fail(CHR_ERR_INVALID, "chr_geometry_create_wide: null traversal BVH");
    return geometry_create(d, w, out);
}
