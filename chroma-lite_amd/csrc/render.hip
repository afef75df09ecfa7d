// render.hip -- the renderer kernels: ray-cast rendering with alpha-depth
// compositing (reference chroma/cuda/render.cu:37-183, driven by
// chroma/gpu/render.py GPURays), the ray transforms (transform.cu:9-48) and the
// hybrid (photon-traced diffuse lighting) renderer (hybrid_render.cu:17-202).
//
// Part of the propagate.hip translation unit (#included at its end): it walks
// the same device BVH (wide_bvh.h) and runs the same photon physics.
//
// Rendering.  The reference walks its BVH with no pruning and keeps, per
// pixel, the alpha_depth nearest hits sorted by distance: each hit found is put
// at searchsorted's position (the first entry >= its distance) of the list, the
// last entry falls off a full list (sorting.h:58-97).  In its traversal order
// (the static DFS order of the reference BVH, the `rank` the wide BVH carries
// per triangle) that leaves the list sorted by (distance ascending, rank
// DESCENDING) with entries of an earlier render (keep_last_render) after every
// new hit of equal distance -- a strict total order, so the list is the top
// alpha_depth of all hits under it whatever order the hits are found in.  Here
// the wide BVH is walked without pruning, every leaf triangle passes the
// reference's own leaf-box slab test first (its ancestors' boxes contain that
// box, and the slab test is monotone in the bounds, so the reference reaches
// exactly the triangles whose leaf box the ray hits), and each hit is inserted
// under that order (ranks kept in a scratch column: earlier entries rank 0,
// new hits rank + 1).
namespace chr {

// render.cu:12-32 (get_color): shading by |cos| of the triangle normal
// r0..r2: the hit's wide triangle record (v0, v1, v2)
__device__ __forceinline__ float4 render_color(V3 dir, float4 r0, float4 r1, float4 r2, uint32_t rgba) {
    const V3 v0 = v3(r0.x, r0.y, r0.z), v1 = v3(r0.w, r1.x, r1.y), v2 = v3(r1.z, r1.w, r2.x);
    const V3 v01 = v1 - v0, v12 = v2 - v1;
    const V3 n = normalize(cross(v01, v12));
    float c = dot(n, -dir);
    if (c < 0.0f) c = -c;
    const uint32_t a0 = 0xFFu & (rgba >> 24), r = 0xFFu & (rgba >> 16), gg = 0xFFu & (rgba >> 8), b = 0xFFu & rgba;
    return make_float4((float)r * c, (float)gg * c, (float)b * c, (float)(255u - a0) / 255.0f);
}

constexpr int RENDER_LDS = 16;   // stack entries per work-item in LDS (deeper ones: private)

__global__ __launch_bounds__(BLOCK) void render_kernel(const DevGeom *__restrict__ gdev, uint32_t nrays,
                                                       const float *origin, const float *direction,
                                                       const uint32_t *colors, uint32_t alpha_depth, uint32_t *pixels,
                                                       float *dx_all, uint32_t *dxlen, float4 *color_all,
                                                       uint32_t bg_color, uint32_t *rank_all) {
    __shared__ uint32_t lds[RENDER_LDS * BLOCK];
    const uint32_t id = blockIdx.x * BLOCK + threadIdx.x;
    if (id >= nrays) return;
    const DevGeom &g = *gdev;
    const V3 o = load3(origin, id), d = load3(direction, id);
    uint32_t n = dxlen[id];
    const V3 noid = v3(-o.x / d.x, -o.y / d.y, -o.z / d.z);
    const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    {
        V3 lo, hi;
        float bd;
        node_bounds(g, gld(g.nodes), lo, hi);
        if (n < 1 && !intersect_box(noid, inv, lo, hi, bd)) {   // render.cu:68-71
            pixels[id] = bg_color;
            return;
        }
    }
    float *dx = dx_all + (size_t)id * alpha_depth;
    float4 *col = color_all + (size_t)id * alpha_depth;
    uint32_t *rk = rank_all + (size_t)id * alpha_depth;
    for (uint32_t i = 0; i < n; ++i) rk[i] = 0u;              // entries of an earlier render
    const RaySlab r = make_slab(o, noid, inv);
    CHR_LDS uint32_t *stk = (CHR_LDS uint32_t *)lds + threadIdx.x;
    uint32_t spill[WIDE_STACK - RENDER_LDS];
    int sp = 0;
    uint32_t node = 0;
    bool have = g.nwnodes != 0;
    while (have) {
        const uint4 *np = g.wnodes + (size_t)g.wstride * node;
        const uint4 h = gld(np), a1 = gld(np + 1), a2 = gld(np + 2), a3 = gld(np + 3), a4 = gld(np + 4),
                    a5 = gld(np + 5);
        const V3 org = v3(__uint_as_float(h.x), __uint_as_float(h.y), __uint_as_float(h.z));
        const float sx = exp_scale(h.w), sy = exp_scale(h.w >> 8), sz = exp_scale(h.w >> 16);
        for (int k = 0; k < 8; ++k) {
            const uint32_t kind = byte_of(a4.z, a4.w, k);
            if (kind == 0) continue;
            const float tnx = __builtin_fmaf(__builtin_fmaf(byte_f(r.negx ? a2.z : a1.x, r.negx ? a2.w : a1.y, k), sx, org.x), r.inx, r.onx);
            const float tfx = __builtin_fmaf(__builtin_fmaf(byte_f(r.negx ? a1.x : a2.z, r.negx ? a1.y : a2.w, k), sx, org.x), r.inx, r.ofx);
            const float tny = __builtin_fmaf(__builtin_fmaf(byte_f(r.negy ? a3.x : a1.z, r.negy ? a3.y : a1.w, k), sy, org.y), r.iny, r.ony);
            const float tfy = __builtin_fmaf(__builtin_fmaf(byte_f(r.negy ? a1.z : a3.x, r.negy ? a1.w : a3.y, k), sy, org.y), r.iny, r.ofy);
            const float tnz = __builtin_fmaf(__builtin_fmaf(byte_f(r.negz ? a3.z : a2.x, r.negz ? a3.w : a2.y, k), sz, org.z), r.inz, r.onz);
            const float tfz = __builtin_fmaf(__builtin_fmaf(byte_f(r.negz ? a2.x : a3.z, r.negz ? a2.y : a3.w, k), sz, org.z), r.inz, r.ofz);
            const float tmin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(tnx, tny), tnz), 0.0f);
            const float tmax = __builtin_fminf(__builtin_fminf(tfx, tfy), tfz);
            if (tmin > tmax) continue;
            const uint32_t off = byte_of(a5.x, a5.y, k);
            if (kind == WIDE_INNER) {
                if (sp < WIDE_STACK) {
                    if (sp < RENDER_LDS) stk[sp * BLOCK] = a4.x + off;
                    else spill[sp - RENDER_LDS] = a4.x + off;
                    sp++;
                }
                continue;
            }
            for (uint32_t j = 0; j < kind; ++j) {
                const float4 *rr = g.wtri + 4 * (size_t)(a4.y + off + j);
                const float4 r0 = gld(rr), r1 = gld(rr + 1), r2 = gld(rr + 2), r3 = gld(rr + 3);
                V3 lo, hi;
                float bd, dist;
                node_bounds(g, make_uint4(__float_as_uint(r2.w), __float_as_uint(r3.x), __float_as_uint(r3.y), 0u), lo, hi);
                if (!intersect_box(noid, inv, lo, hi, bd)) continue;   // the reference's leaf node test
                if (!intersect_record(o, d, r0, r1, r2, dist))
                    continue;
                const uint32_t tid = __float_as_uint(r2.y), rank = __float_as_uint(r2.z) + 1u;
                // position under (distance asc, rank desc); a full list drops its last entry
                uint32_t pos = n;
                for (uint32_t i = 0; i < n; ++i) {
                    const float e = dx[i];
                    if (e > dist || (e == dist && rk[i] < rank)) { pos = i; break; }
                }
                if (pos > alpha_depth - 1) continue;
                const uint32_t last = n < alpha_depth ? n : alpha_depth - 1;
                for (uint32_t i = last; i > pos; --i) {
                    dx[i] = dx[i - 1];
                    col[i] = col[i - 1];
                    rk[i] = rk[i - 1];
                }
                dx[pos] = dist;
                col[pos] = render_color(d, r0, r1, r2, gld(colors + tid));
                rk[pos] = rank;
                if (n < alpha_depth) n++;
            }
        }
        if (sp == 0) break;
        sp--;
        node = sp < RENDER_LDS ? stk[sp * BLOCK] : spill[sp - RENDER_LDS];
    }
    if (n < 1) {
        pixels[id] = bg_color;
        return;
    }
    dxlen[id] = n;
    // render.cu:150-179 (a*b + c contracted as nvcc does)
    float scale = 1.0f, fr = 0.0f, fg = 0.0f, fb = 0.0f;
    for (uint32_t i = 0; i < n; ++i) {
        const float4 c = col[i];
        const float alpha = c.w;
        fr = __builtin_fmaf(scale * c.x, alpha, fr);
        fg = __builtin_fmaf(scale * c.y, alpha, fg);
        fb = __builtin_fmaf(scale * c.z, alpha, fb);
        scale *= (1.0f - alpha);
    }
    const float alpha = (float)((double)((bg_color & 0xFF000000u) >> 24) / 255.0);
    fr = __builtin_fmaf(scale * (float)((bg_color & 0xFF0000u) >> 16), alpha, fr);
    fg = __builtin_fmaf(scale * (float)((bg_color & 0xFF00u) >> 8), alpha, fg);
    fb = __builtin_fmaf(scale * (float)(bg_color & 0xFFu), alpha, fb);
    scale *= (1.0f - alpha);
    const uint32_t a = n < alpha_depth ? chr_sat_u32(__builtin_floorf(255.0f * (1.0f - scale))) : 255u;
    const uint32_t red = chr_sat_u32(__builtin_floorf(fr / (1.0f - scale)));
    const uint32_t green = chr_sat_u32(__builtin_floorf(fg / (1.0f - scale)));
    const uint32_t blue = chr_sat_u32(__builtin_floorf(fb / (1.0f - scale)));
    pixels[id] = a << 24 | red << 16 | green << 8 | blue;
}

// transform.cu:9-48
__global__ __launch_bounds__(BLOCK) void transform_kernel(uint32_t n, float *a, int mode, float phi, V3 axis, V3 v) {
    const uint32_t id = blockIdx.x * BLOCK + threadIdx.x;
    if (id >= n) return;
    V3 x = load3(a, id);
    if (mode == 0) {
        x += v;                                   // translate
    } else if (mode == 1) {
        x = rotate(x, phi, axis);                 // rotate
    } else {
        x -= v;                                   // rotate_around_point
        x = rotate(x, phi, axis);
        x += v;
    }
    store3(a, id, x);
}

// hybrid_render.cu:17-55: propagate until the first diffuse reflection
__device__ void to_diffuse(const DevGeom &g, Photon &p, State &s, chr_xorwow &rng, int max_steps, WStack &wst,
                           uint32_t &overflow) {
    Stack st;
    st.lds = nullptr;
    WalkCounts cnt;
    int steps = 0;
    while (steps < max_steps) {
        steps++;
        fill_state<8, kWalkSched, false>(g, s, p, st, wst, overflow, cnt);
        if (p.last_hit == -1) break;
        int command = propagate_to_boundary(g, p, s, rng, 0, 0);
        if (command == BREAK) break;
        if (command == CONTINUE) continue;
        if (s.surface_index != -1) {
            command = propagate_at_surface(g, p, s, rng, 0);
            if (p.history & CHR_REFLECT_DIFFUSE) break;
            if (command == BREAK) break;
            if (command == CONTINUE) continue;
        }
        propagate_at_boundary(p, s, rng);
    }
}

#define CHR_HYBRID_WSTACK                                                          \
    __shared__ uint32_t lds_stack[lds_words(kWalkSched) * BLOCK];                 \
    WStack wst;                                                                    \
    uint2 wspill[WIDE_STACK - WIDE_LDS];                                           \
    wst.spill = wspill;                                                            \
    wst.sstride = 1;                                                               \
    wst.node = (CHR_LDS uint32_t *)(lds_stack + threadIdx.x);                      \
    wst.dist = (CHR_LDS float *)(lds_stack + WIDE_LDS * BLOCK + threadIdx.x);      \
    wst.leafq = nullptr

// float adds of the per-triangle lookup (the reference's fAtomicAdd loop)
__device__ __forceinline__ void lookup_add(float *base, uint32_t tri, V3 v) {
    atomicAdd(base + 3 * (size_t)tri, v.x);
    atomicAdd(base + 3 * (size_t)tri + 1, v.y);
    atomicAdd(base + 3 * (size_t)tri + 2, v.z);
}

// hybrid_render.cu:61-131
__global__ __launch_bounds__(BLOCK) void update_xyz_lookup_kernel(const DevGeom *__restrict__ gdev,
                                                                  const float *vertices, const uint32_t *triangles,
                                                                  int nthreads, int total_threads, int offset, V3 position,
                                                                  uint32_t *rng_states, uint32_t nslots,
                                                                  float wavelength, V3 xyz, float *lookup1,
                                                                  float *lookup2, int max_steps, uint32_t *counters) {
    CHR_HYBRID_WSTACK;
    const int kid = blockIdx.x * BLOCK + threadIdx.x;
    const int id = kid + offset;
    if (kid >= nthreads || id >= total_threads) return;
    const DevGeom &g = *gdev;
    PropagateArgs ra{};
    ra.rng = rng_states;
    ra.nslots = nslots;
    chr_xorwow rng;
    load_rng(ra, (uint32_t)kid, rng);
    // get_triangle (geometry.h): the mesh's own vertices
    const V3 v0 = load3(vertices, triangles[3 * (size_t)id]), v1 = load3(vertices, triangles[3 * (size_t)id + 1]),
             v2 = load3(vertices, triangles[3 * (size_t)id + 2]);
    const float a = chr_uniform01(&rng);
    const float b = chr_uniform(&rng, 0.0f, 1.0f - a);
    const float c = (1.0f - a) - b;
    // a*v0 + b*v1 + c*v2 - position, contracted as nvcc does: fma(c, v2, fma(b, v1, a*v0))
    V3 dir = v3(__builtin_fmaf(c, v2.x, __builtin_fmaf(b, v1.x, a * v0.x)),
                __builtin_fmaf(c, v2.y, __builtin_fmaf(b, v1.y, a * v0.y)),
                __builtin_fmaf(c, v2.z, __builtin_fmaf(b, v1.z, a * v0.z))) - position;
    dir /= norm(dir);
    uint32_t overflow = 0;
    WalkCounts cnt;
    float distance;
    const int rec = intersect_wide_sched<false, 2>(g, position, dir, distance, -1, wst, overflow, cnt);
    const int hit = rec == -1 ? -1 : (int)__float_as_uint(gld(g.wtri + 4 * (size_t)rec + 2).y);   // the record's triangle
    if (hit == id) {
        const V3 nrm = normalize(cross(v1 - v0, v2 - v1));
        float cos_theta = dot(nrm, -dir);
        if (cos_theta < 0.0f) cos_theta = dot(-nrm, -dir);
        Photon p;
        p.pos = position;
        p.dir = dir;
        p.wavelength = wavelength;
        p.pol = uniform_sphere(rng);
        p.last_hit = -1;
        p.time = 0.0f;
        p.history = 0;
        p.weight = 1.0f;
        State s;
        to_diffuse(g, p, s, rng, max_steps, wst, overflow);
        // (a diffuse reflection on an analytic wire plane has no triangle: last_hit -2; the
        // reference indexes the lookup with it, out of bounds -- skipped here)
        if ((p.history & CHR_REFLECT_DIFFUSE) && p.last_hit >= 0)
            lookup_add(s.inside_to_outside ? lookup1 : lookup2, (uint32_t)p.last_hit, xyz * cos_theta);
    }
    store_rng(ra, (uint32_t)kid, rng);
    if (overflow && counters) atomicAdd(counters, overflow);
}

// hybrid_render.cu:133-166
__global__ __launch_bounds__(BLOCK) void update_xyz_image_kernel(const DevGeom *__restrict__ gdev, int nthreads,
                                                                 uint32_t *rng_states, uint32_t nslots,
                                                                 const float *positions, const float *directions,
                                                                 float wavelength, V3 xyz, const float *lookup1,
                                                                 const float *lookup2, float *image,
                                                                 int nlookup_calls, int max_steps, uint32_t *counters) {
    CHR_HYBRID_WSTACK;
    const int id = blockIdx.x * BLOCK + threadIdx.x;
    if (id >= nthreads) return;
    const DevGeom &g = *gdev;
    PropagateArgs ra{};
    ra.rng = rng_states;
    ra.nslots = nslots;
    chr_xorwow rng;
    load_rng(ra, (uint32_t)id, rng);
    Photon p;
    p.pos = load3(positions, id);
    p.dir = load3(directions, id);
    p.dir /= norm(p.dir);
    p.wavelength = wavelength;
    p.pol = uniform_sphere(rng);
    p.last_hit = -1;
    p.time = 0.0f;
    p.history = 0;
    p.weight = 1.0f;
    State s;
    uint32_t overflow = 0;
    to_diffuse(g, p, s, rng, max_steps, wst, overflow);
    if ((p.history & CHR_REFLECT_DIFFUSE) && p.last_hit >= 0) {
        const float *lk = (s.inside_to_outside ? lookup1 : lookup2) + 3 * (size_t)p.last_hit;
        // image += xyz * lookup / nlookup_calls (float3 ops of linalg.h, left to right)
        const V3 add = v3(xyz.x * lk[0], xyz.y * lk[1], xyz.z * lk[2]) / (float)nlookup_calls;
        store3(image, (uint32_t)id, load3(image, id) + add);
    }
    store_rng(ra, (uint32_t)id, rng);
    if (overflow && counters) atomicAdd(counters, overflow);
}

// hybrid_render.cu:168-200
__global__ __launch_bounds__(BLOCK) void process_image_kernel(int nthreads, const float *image, uint32_t *pixels,
                                                              int nimages) {
    const int id = blockIdx.x * BLOCK + threadIdx.x;
    if (id >= nthreads) return;
    V3 rgb = load3(image, id) / (float)nimages;
    rgb.x = rgb.x < 0.0f ? 0.0f : (rgb.x > 1.0f ? 1.0f : rgb.x);
    rgb.y = rgb.y < 0.0f ? 0.0f : (rgb.y > 1.0f ? 1.0f : rgb.y);
    rgb.z = rgb.z < 0.0f ? 0.0f : (rgb.z > 1.0f ? 1.0f : rgb.z);
    const uint32_t r = chr_sat_u32(__builtin_floorf(rgb.x * 255.0f));
    const uint32_t gg = chr_sat_u32(__builtin_floorf(rgb.y * 255.0f));
    const uint32_t b = chr_sat_u32(__builtin_floorf(rgb.z * 255.0f));
    pixels[id] = 255u << 24 | r << 16 | gg << 8 | b;
}

}  // namespace chr

using namespace chr;

static int render_rank_scratch(size_t bytes, uint32_t **out) {
    static thread_local Scratch s[16];
    int dev = 0;
    CHR_HIP_CHECK(hipGetDevice(&dev));
    Scratch &x = s[dev & 15];
    if (x.bytes < bytes) {
        if (x.ptr) CHR_HIP_CHECK(hipFree(x.ptr));
        x.ptr = nullptr;
        CHR_HIP_CHECK(hipMalloc(&x.ptr, bytes));
        x.bytes = bytes;
    }
    *out = (uint32_t *)x.ptr;
    return CHR_OK;
}

extern "C" int chr_render(const chr_geometry *g, uint32_t nrays, const float *d_pos, const float *d_dir,
                          const uint32_t *d_colors, uint32_t alpha_depth, uint32_t *d_pixels, float *d_dx,
                          uint32_t *d_dxlen, float *d_color, uint32_t bg_color, void *stream) {
    if (!g || !d_pos || !d_dir || !d_colors || !d_pixels || !d_dx || !d_dxlen || !d_color)
        return chr::fail(CHR_ERR_INVALID, "chr_render: null argument");
    if (alpha_depth < 1) return chr::fail(CHR_ERR_INVALID, "chr_render: alpha_depth must be >= 1");
    if (g->dev.nwnodes == 0) return chr::fail(CHR_ERR_INVALID, "chr_render: the geometry has no traversal BVH");
    if (nrays == 0) return CHR_OK;
    uint32_t *rk = nullptr;
    if (int rc = render_rank_scratch((size_t)nrays * alpha_depth * 4, &rk)) return rc;
    hipLaunchKernelGGL(render_kernel, dim3(grid_for(nrays)), dim3(BLOCK), 0, (hipStream_t)stream,
                       (const DevGeom *)g->d_dev, nrays, d_pos, d_dir, d_colors, alpha_depth, d_pixels, d_dx, d_dxlen,
                       (float4 *)d_color, bg_color, rk);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

static int transform(uint32_t n, float *d_a, int mode, float phi, V3 axis, V3 v, void *stream) {
    if (!d_a) return chr::fail(CHR_ERR_INVALID, "transform: null argument");
    if (n == 0) return CHR_OK;
    hipLaunchKernelGGL(transform_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, (hipStream_t)stream, n, d_a, mode, phi,
                       axis, v);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_transform_translate(uint32_t n, float *d_a, float vx, float vy, float vz, void *stream) {
    return transform(n, d_a, 0, 0.0f, V3{0.0f, 0.0f, 0.0f}, V3{vx, vy, vz}, stream);
}

extern "C" int chr_transform_rotate(uint32_t n, float *d_a, float phi, float ax, float ay, float az, void *stream) {
    return transform(n, d_a, 1, phi, V3{ax, ay, az}, V3{0.0f, 0.0f, 0.0f}, stream);
}

extern "C" int chr_transform_rotate_around_point(uint32_t n, float *d_a, float phi, float ax, float ay, float az,
                                                 float px, float py, float pz, void *stream) {
    return transform(n, d_a, 2, phi, V3{ax, ay, az}, V3{px, py, pz}, stream);
}

extern "C" int chr_hybrid_update_xyz_lookup(const chr_geometry *g, const float *d_vertices, const uint32_t *d_triangles,
                                            int32_t nthreads, int32_t total_threads,
                                            int32_t offset, const float *position, uint32_t *d_rng_states,
                                            uint32_t rng_nslots, float wavelength, const float *xyz,
                                            float *d_lookup1, float *d_lookup2, int32_t max_steps, void *stream) {
    if (!g || !d_vertices || !d_triangles || !position || !d_rng_states || !xyz || !d_lookup1 || !d_lookup2)
        return chr::fail(CHR_ERR_INVALID, "chr_hybrid_update_xyz_lookup: null argument");
    if (g->dev.nwnodes == 0) return chr::fail(CHR_ERR_INVALID, "chr_hybrid_update_xyz_lookup: no traversal BVH");
    if (nthreads <= 0) return CHR_OK;
    if ((uint32_t)nthreads > rng_nslots)
        return chr::fail(CHR_ERR_INVALID, "chr_hybrid_update_xyz_lookup: %d threads, %u rng states", nthreads, rng_nslots);
    if (total_threads > (int32_t)g->dev.ntriangles)
        return chr::fail(CHR_ERR_INVALID, "chr_hybrid_update_xyz_lookup: %d lookup entries, %u triangles",
                         total_threads, g->dev.ntriangles);
    hipLaunchKernelGGL(update_xyz_lookup_kernel, dim3(grid_for((uint32_t)nthreads)), dim3(BLOCK), 0, (hipStream_t)stream,
                       (const DevGeom *)g->d_dev, d_vertices, d_triangles, nthreads, total_threads, offset,
                       V3{position[0], position[1], position[2]},
                       d_rng_states, rng_nslots, wavelength, V3{xyz[0], xyz[1], xyz[2]}, d_lookup1, d_lookup2, max_steps,
                       (uint32_t *)nullptr);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_hybrid_update_xyz_image(const chr_geometry *g, int32_t nthreads, uint32_t *d_rng_states,
                                           uint32_t rng_nslots, const float *d_positions, const float *d_directions,
                                           float wavelength, const float *xyz, const float *d_lookup1,
                                           const float *d_lookup2, float *d_image, int32_t nlookup_calls,
                                           int32_t max_steps, void *stream) {
    if (!g || !d_rng_states || !d_positions || !d_directions || !xyz || !d_lookup1 || !d_lookup2 || !d_image)
        return chr::fail(CHR_ERR_INVALID, "chr_hybrid_update_xyz_image: null argument");
    if (g->dev.nwnodes == 0) return chr::fail(CHR_ERR_INVALID, "chr_hybrid_update_xyz_image: no traversal BVH");
    if (nthreads <= 0) return CHR_OK;
    if ((uint32_t)nthreads > rng_nslots)
        return chr::fail(CHR_ERR_INVALID, "chr_hybrid_update_xyz_image: %d threads, %u rng states", nthreads, rng_nslots);
    hipLaunchKernelGGL(update_xyz_image_kernel, dim3(grid_for((uint32_t)nthreads)), dim3(BLOCK), 0, (hipStream_t)stream,
                       (const DevGeom *)g->d_dev, nthreads, d_rng_states, rng_nslots, d_positions, d_directions,
                       wavelength, V3{xyz[0], xyz[1], xyz[2]}, d_lookup1, d_lookup2, d_image, nlookup_calls, max_steps,
                       (uint32_t *)nullptr);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}

extern "C" int chr_hybrid_process_image(int32_t nthreads, const float *d_image, uint32_t *d_pixels, int32_t nimages,
                                        void *stream) {
    if (!d_image || !d_pixels) return chr::fail(CHR_ERR_INVALID, "chr_hybrid_process_image: null argument");
    if (nthreads <= 0) return CHR_OK;
    hipLaunchKernelGGL(process_image_kernel, dim3(grid_for((uint32_t)nthreads)), dim3(BLOCK), 0, (hipStream_t)stream,
                       nthreads, d_image, d_pixels, nimages);
    CHR_HIP_CHECK(hipGetLastError());
    return CHR_OK;
}
