/* chroma_amd.h -- C ABI of the MI355X-native Chroma propagator (libchroma_amd.so).
 *
 * Every entry point replaces one thing the reference binds through PyCUDA
 * (a JIT-compiled `extern "C" __global__` kernel launched from Python, or a
 * make_gpu_struct() upload).  The "replaces" line on each declaration cites the
 * reference interface (paths relative to youngsm/chroma-lite).
 *
 * Conventions
 *  - plain C types only; no torch / HIP types in the signatures.  `stream` is a
 *    hipStream_t passed as void* (NULL = default stream).
 *  - pointers named d_* are DEVICE pointers (e.g. torch.Tensor.data_ptr()),
 *    pointers named h_* are host pointers.
 *  - photon vectors (pos/dir/pol) are float3-packed: 3 floats per photon,
 *    exactly the reference's ga.vec.float3 arrays (chroma/gpu/photon.py:46-48).
 *  - every function returns 0 on success or a nonzero chr_status; the message
 *    of the last failure on the calling thread is chr_last_error().
 *  - all launches are asynchronous on `stream` unless documented otherwise;
 *    functions that return a count to the host synchronise the stream.
 */
#ifndef CHROMA_AMD_H
#define CHROMA_AMD_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum chr_status {
    CHR_OK = 0,
    CHR_ERR_INVALID = 1,     /* bad argument (reference: ValueError / assert) */
    CHR_ERR_HIP = 2,         /* HIP runtime error (reference: pycuda LogicError/LaunchError) */
    CHR_ERR_NOMEM = 3,
    CHR_ERR_STACK = 4        /* BVH stack overflow (reference: printf in mesh.h:111-114) */
};

/* photon history bits as stored on the device (reference photon.h:53-68).
 * NOTE the reference keeps history in an unsigned short on the device, so
 * NAN_ABORT is bit 15 there (and any propagate clears bits 16..31). */
enum chr_history {
    CHR_NO_HIT = 1u << 0, CHR_BULK_ABSORB = 1u << 1, CHR_SURFACE_DETECT = 1u << 2,
    CHR_SURFACE_ABSORB = 1u << 3, CHR_RAYLEIGH_SCATTER = 1u << 4, CHR_REFLECT_DIFFUSE = 1u << 5,
    CHR_REFLECT_SPECULAR = 1u << 6, CHR_SURFACE_REEMIT = 1u << 7, CHR_SURFACE_TRANSMIT = 1u << 8,
    CHR_BULK_REEMIT = 1u << 9, CHR_CHERENKOV = 1u << 10, CHR_SCINTILLATION = 1u << 11,
    CHR_NAN_ABORT = 1u << 15
};

/* surface models (reference geometry_types.h:22) */
enum chr_surface_model { CHR_SURFACE_DEFAULT = 0, CHR_SURFACE_COMPLEX = 1, CHR_SURFACE_WLS = 2,
                         CHR_SURFACE_DICHROIC = 3, CHR_SURFACE_ANGULAR = 4 };

/* ---------------------------------------------------------------- geometry
 * Host-side description of a flattened, BVH-indexed geometry.  All tables are
 * sampled on one wavelength grid (wavelength_start + i*wavelength_step,
 * i < wavelength_n) and one time grid, as GPUGeometry does
 * (chroma/gpu/geometry.py:44-107).  EVERY table pointer must address n+1
 * floats: the last element duplicates element n-1 (the reference's
 * interp_property reads fp[n] at x == last grid point, geometry.h:61-74).
 */
typedef struct chr_material_desc {         /* reference struct Material, geometry_types.h:4-20 */
    uint32_t num_comp;
    const float *refractive_index;          /* [wavelength_n+1] */
    const float *absorption_length;
    const float *scattering_length;
    const float *comp_reemission_prob;      /* [num_comp][wavelength_n+1] */
    const float *comp_reemission_wvl_cdf;   /* [num_comp][wavelength_n+1] */
    const float *comp_reemission_time_cdf;  /* [num_comp][time_n+1] */
    const float *comp_absorption_length;    /* [num_comp][wavelength_n+1] */
} chr_material_desc;

typedef struct chr_surface_desc {          /* reference struct Surface, geometry_types.h:60-79 */
    int32_t present;                        /* 0: NULL slot (the `None` surface) */
    uint32_t model;                         /* chr_surface_model */
    uint32_t transmissive;
    float thickness;
    const float *detect, *absorb, *reemit, *reflect_diffuse, *reflect_specular,
                *eta, *k, *reemission_cdf;  /* [wavelength_n+1] each */
    uint32_t dichroic_nangles;              /* 0: no DichroicProps */
    const float *dichroic_angles;           /* [nangles] */
    const float *dichroic_reflect;          /* [nangles][wavelength_n+1] */
    const float *dichroic_transmit;         /* [nangles][wavelength_n+1] */
    uint32_t angular_nangles;               /* 0: no AngularProps */
    const float *angular_angles, *angular_transmit, *angular_reflect_specular,
                *angular_reflect_diffuse;   /* [nangles] */
} chr_surface_desc;

typedef struct chr_wireplane_desc {        /* reference struct WirePlane, geometry_types.h:42-58 */
    float origin[3], u[3], v[3];
    float pitch, radius, umin, umax, vmin, vmax, v0;
    int32_t surface_index, material_outer_index, material_inner_index;
    uint32_t color;
} chr_wireplane_desc;

typedef struct chr_geometry_desc {         /* reference struct Geometry, geometry_types.h:124-139 */
    uint32_t nvertices, ntriangles, nnodes;
    uint32_t nmaterials, nsurfaces, nwireplanes;
    const float *h_vertices;                /* [nvertices*3] */
    const uint32_t *h_triangles;            /* [ntriangles*3] */
    const uint32_t *h_material_codes;       /* [ntriangles]: m1<<24 | m2<<16 | surf<<8 (gpu/geometry.py:401-404) */
    const uint32_t *h_nodes;                /* [nnodes*4] packed uint4 BVH nodes (bvh/bvh.py:106-195) */
    float world_origin[3];
    float world_scale;
    uint32_t wavelength_n; float wavelength_start, wavelength_step;
    uint32_t time_n; float time_start, time_step;
    const chr_material_desc *materials;
    const chr_surface_desc *surfaces;
    const chr_wireplane_desc *wireplanes;
} chr_geometry_desc;

typedef struct chr_geometry chr_geometry;  /* opaque device-resident geometry */

/* replaces: GPUGeometry.__init__ device uploads (chroma/gpu/geometry.py:14-526).
 * Copies everything to HBM of the current device, builds the traversal layout.
 * Synchronous. */
int chr_geometry_create(const chr_geometry_desc *desc, chr_geometry **out);
int chr_geometry_destroy(chr_geometry *g);
/* bytes of HBM held by the geometry (reference: GPUGeometry.device_usage_str) */
int chr_geometry_device_bytes(const chr_geometry *g, uint64_t *bytes);
/* words (4 B) of the physics tables and records: the hot part the step kernels
 * copy to LDS when it fits (property tables, identical tables stored once, the
 * material / surface records) and the whole (+ re-emission time CDFs and their
 * bucket indexes, read from HBM).  No reference counterpart (diagnostic). */
int chr_geometry_phys_words(const chr_geometry *g, uint32_t *hot_words, uint32_t *total_words);

/* ----------------------------------------------------------------- photons */
typedef struct chr_photons {               /* reference GPUPhotons arrays, photon.py:46-62 */
    float *d_pos, *d_dir, *d_pol;          /* float3-packed [n*3] */
    float *d_wavelengths, *d_t, *d_weights;
    uint32_t *d_flags;
    int32_t *d_last_hit_triangles;
    uint32_t *d_evidx;
} chr_photons;

/* ---------------------------------------------------------------- random */
/* RNG slot states: 6 x u32 per slot, SoA (word k of slot s at d_states[k*nslots+s]).
 * replaces: get_rng_states / init_rng (chroma/gpu/tools.py:117-145):
 * curand_init(seed, subsequence = slot, offset) for every slot. */
int chr_init_rng(uint32_t *d_states, uint32_t nslots, uint64_t seed, uint64_t offset, void *stream);
/* extension for photon-sharded runs: slot s = curand_init(seed, first_subsequence + s, offset)
 * (first_subsequence + nslots <= 2^32); chr_init_rng is first_subsequence = 0. */
int chr_init_rng_subseq(uint32_t *d_states, uint32_t nslots, uint64_t seed, uint64_t first_subsequence,
                        uint64_t offset, void *stream);
/* copy slot states to the host (tests; 6*nslots words, SoA) */
int chr_rng_download(const uint32_t *d_states, uint32_t nslots, uint32_t *h_out, void *stream);

/* -------------------------------------------------------------- propagate */
/* replaces: the `propagate` kernel (chroma/cuda/propagate.cu:254-366), one
 * chunk launch: slots [0, nthreads), photon = d_input_queue[first_photon + slot].
 * Survivors are appended to d_output_queue in input order (stable; the
 * reference's warp-atomic order is nondeterministic) and d_output_queue[0]
 * counts them (+1, photon.py:248-250).  d_scratch must hold
 * chr_propagate_scratch_words(nthreads) u32 words. */
uint64_t chr_propagate_scratch_words(uint32_t nthreads);
int chr_propagate_chunk(const chr_geometry *g, const chr_photons *ph, uint32_t *d_rng_states,
                        uint32_t rng_nslots, int32_t first_photon, int32_t nthreads,
                        const uint32_t *d_input_queue, uint32_t *d_output_queue,
                        int32_t max_steps, int32_t use_weights, int32_t scatter_first,
                        uint32_t *d_scratch, void *stream);

typedef struct chr_propagate_stats {
    uint32_t steps_run;         /* host-loop steps executed */
    uint32_t launches;          /* chunk launches */
    uint32_t final_alive;       /* photons still in the queue at exit */
    uint32_t stack_overflows;   /* traversals that exceeded the 1000-entry stack */
    double kernel_ms;           /* summed device time of the propagate kernels (HIP events; device-driven
                                   propagates record them only with CHR_SLOT_TIMING=1, else 0) */
    uint64_t nodes_visited;     /* BVH nodes / triangles / walks: filled only by the counting */
    uint64_t triangles_tested;  /* kernel variant (CHR_PROPAGATE_VARIANT=5), zero otherwise */
    uint64_t traversals;
    uint64_t wave_node_steps;     /* node / triangle steps executed per wave (SIMD efficiency = */
    uint64_t wave_triangle_steps; /* nodes_visited / (64 * wave_node_steps)); counting variant only */
    uint64_t wave_fill_cycles;    /* s_memtime cycles waves spent in fill_state (traversal) and in */
    uint64_t wave_step_cycles;    /* whole photon step loops; counting variant only */
    double trace_ms;              /* device time of the BVH-walk kernel (trace_kernel) alone, HIP events */
    uint32_t trace_launches;      /* one-step launches walked by trace_kernel */
    uint32_t reserved;
    uint64_t trace_rays;          /* queued photons handed to those launches */
    uint32_t trace_ms_n;          /* entries of trace_launch_ms filled (first CHR_TRACE_MS_MAX launches) */
    float trace_launch_ms[32];    /* device time of each trace_kernel launch, in order */
    uint32_t flat_walks;          /* walks with a direction component of non-finite reciprocal (the reference's
                                     slab test then skips that axis) done by trace_kernel (flat-axis slab test) */
    uint32_t flat_walks_whole;    /* such walks done by the multi-step (tail) kernel */
    uint32_t tail_photons;        /* photons handed to the multi-step (tail) launch (nsteps policy) */
    double tail_ms;               /* device time of that launch (HIP events; CHR_SLOT_TIMING=1, else 0) */
    uint32_t tail_max_steps;      /* most steps one photon ran in the tail launch */
    uint32_t tail_slowest_steps;  /* steps of the photon that took longest in the tail launch */
    uint64_t tail_max_cycles;     /* that photon's time in ticks of the 100 MHz s_memrealtime clock */
    uint32_t tail_long_photons;   /* photons of > 64 steps in the tail launch, and summed over them: */
    uint32_t reserved2;
    uint64_t tail_long_steps;     /*   steps, */
    uint64_t tail_long_ticks;     /*   100 MHz ticks from load to write-back, */
    uint64_t tail_long_walk_ticks;        /*   ticks in the BVH walk (wave-adaptive tail kernel), */
    uint64_t tail_long_walk_iterations;   /*   and dependent walk iterations */
    uint32_t host_syncs;          /* waits that drain the stream (the host reads the survivor count): one
                                     per host step when host-driven, 1 when the steps are device-driven */
    uint32_t tail_long_paired_steps;  /* the long photons' steps whose walk had a tester wave (walk_pair) */
    uint32_t trace_launch_rays[32];   /* queued photons of each trace_kernel launch, in order */
} chr_propagate_stats;
#define CHR_TRACE_MS_MAX 32

/* Resources of the kernels on the default propagate path, from the code object
 * (hipFuncGetAttributes): which = 0 trace_kernel (BVH walk of one-step launches),
 * 1 shade_kernel, 2 the tail's group-walk kernel, 3 the fused step kernel.
 * No reference counterpart (bench diagnostics). */
typedef struct chr_kernel_attr {
    uint64_t private_bytes;     /* scratch per work-item (0: no private segment) */
    uint64_t lds_bytes;         /* static LDS per workgroup */
    int32_t vgprs;              /* architected VGPRs per work-item */
    int32_t max_threads;        /* max workgroup size */
    char name[96];
} chr_kernel_attr;
int chr_kernel_info(int32_t which, chr_kernel_attr *out);
/* Diagnostic (no reference counterpart): the tail's lone-photon walk timed in
 * isolation, walker 0 = walk_lone on one wave, 1 = the pair walk (one wave walks,
 * a second wave of the workgroup tests the triangles), 2 = the pair walk with a
 * 2-poll handshake budget, so handshakes are lost and the tail kernel's recovery
 * (the walk again with walk_lone, no more pairing in that workgroup) runs; each
 * lost handshake adds 1 << 20 to the last word; 3 = walk_up from an arbitrary
 * node (ray r: (r * 2654435761) mod nodes), 4 = walk_up from the leaf node of a
 * given record (d_rays then n x 8 words: + the record index), 5 = the grouped
 * walk's climb (one 64-lane segment) from walker 3's start, 7 = walker 3 with the
 * start node's ancestors read beforehand (the tail's prefetch).  nwaves workgroups; workgroup
 * w walks rays w, w + nwaves, ... each reps times in a row.  d_rays: n x 7 floats
 * (origin, direction, last hit triangle id as int bits); d_out: n x reps x 4 words
 * (record index or -1, iterations, 100 MHz ticks, shader-clock cycles of the walk)
 * + 1 word, the stack overflows (low 20 bits, must read 0) + lost handshakes << 20. */
int chr_walk_lone_timing(const chr_geometry *g, const float *d_rays, uint32_t n, uint32_t reps,
                         uint32_t nwaves, int32_t walker, uint32_t *d_out, void *stream);

/* replaces: GPUPhotons.propagate host loop (chroma/gpu/photon.py:226-293) for
 * track=False: queue setup (clones interleaved, 242-250), the nsteps policy
 * (261-264), chunk_iterator chunking (tools.py:159-180), queue swap and the
 * per-step survivor count (277-286).  Synchronous. */
int chr_propagate(const chr_geometry *g, const chr_photons *ph, uint32_t nphotons,
                  uint32_t true_nphotons, uint32_t ncopies,
                  uint32_t *d_rng_states, uint32_t rng_nslots,
                  int32_t nthreads_per_block, int32_t max_blocks, int32_t max_steps,
                  int32_t use_weights, int32_t scatter_first,
                  chr_propagate_stats *stats, void *stream);

/* replaces: a sequence of GPUPhotons.propagate calls sharing one rng_states
 * (the event loop of Simulation.simulate, chroma/sim.py:116-160, one propagate
 * per event): batch i = photons phs[i] (nphotons[i] = true_nphotons[i] *
 * ncopies[i]), propagated in order with the same RNG slot states and the same
 * launch shape.  Results (photons, RNG states) are bit-identical to nbatch
 * chr_propagate calls; the multi-step tail of batch i runs on a second stream
 * while batch i+1 queues, bins and walks its first step (which needs no RNG),
 * and batch i+1's first RNG use waits for that tail.  stats: nbatch entries
 * (or NULL).  Batches whose photon arrays overlap are serialised.  Synchronous. */
int chr_propagate_batches(const chr_geometry *g, const chr_photons *phs, const uint32_t *nphotons,
                          const uint32_t *true_nphotons, const uint32_t *ncopies, uint32_t nbatch,
                          uint32_t *d_rng_states, uint32_t rng_nslots,
                          int32_t nthreads_per_block, int32_t max_blocks, int32_t max_steps,
                          int32_t use_weights, int32_t scatter_first,
                          chr_propagate_stats *stats, void *stream);

/* ------------------------------------------------------------ selection */
/* replaces: count_photon_hits + copy_photon_hits (propagate.cu:172-251),
 * driven by GPUPhotons.get_flat_hits (photon.py:141-209).  Hits are compacted
 * in ascending photon order.  Pass d_out.* = NULL to only count.  *nhits is
 * written on the host (synchronises). */
int chr_photon_hits(const chr_photons *ph, int32_t start_photon, int32_t nphotons,
                    uint32_t detection_state, const uint32_t *d_solid_map,
                    const int32_t *d_solid_id_to_channel_index,
                    const chr_photons *d_out, int32_t *d_out_channels,
                    uint32_t *nhits, void *stream);
/* replaces: count_photons + copy_photons (propagate.cu:70-139) = GPUPhotons.select */
int chr_select_photons(const chr_photons *ph, int32_t start_photon, int32_t nphotons,
                       uint32_t target_flag, const chr_photons *d_out, uint32_t *nselected,
                       void *stream);
/* replaces: copy_photon_queue (propagate.cu:141-169): out[i] = in[queue[i]], i in [first, first+n) */
int chr_copy_photon_queue(const chr_photons *ph, int32_t first_photon, int32_t nphotons,
                          const uint32_t *d_queue, const chr_photons *d_out, void *stream);
/* replaces: photon_duplicate (propagate.cu:29-68): copy photon i to i + stride*c, c=1..copies.
 * evidx must be allocated nphotons*(copies+1) (the reference allocates only n: photon.py:62). */
int chr_photon_duplicate(const chr_photons *ph, int32_t first_photon, int32_t nphotons,
                         int32_t copies, int32_t stride, void *stream);

/* replaces: distance_to_mesh test kernel (chroma/cuda/mesh.h:131-159).
 * d_distance[i] is written only when ray i hits (reference semantics). */
int chr_distance_to_mesh(const chr_geometry *g, uint32_t n, const float *d_origin,
                         const float *d_direction, float *d_distance, void *stream);

/* ------------------------------------------------------------- BVH build */
/* replaces: make_recursive_grid_bvh (chroma/bvh/grid.py:11-95) with its GPU
 * helpers create_leaf_nodes/make_leaves, merge_nodes_detailed/make_parents_detailed,
 * concatenate_layers/copy_and_offset and collapse_chains/collapse_child
 * (chroma/gpu/bvh.py:18-130, chroma/cuda/bvh.cu:148-384,530-543), on the host.
 * Leaves with equal Morton codes keep triangle order (stable sort; the
 * reference's numpy quicksort is unstable).  The result is an opaque handle:
 * query sizes with chr_bvh_result_info, copy out with chr_bvh_result_copy. */
typedef struct chr_bvh_result chr_bvh_result;
int chr_bvh_build_grid(const float *h_vertices, uint32_t nvertices,
                       const uint32_t *h_triangles, uint32_t ntriangles,
                       int32_t target_degree, chr_bvh_result **out);
int chr_bvh_result_info(const chr_bvh_result *r, uint32_t *nnodes, uint32_t *nlayers,
                        float *world_origin /*[3]*/, float *world_scale);
int chr_bvh_result_copy(const chr_bvh_result *r, uint32_t *h_nodes /*[nnodes*4]*/,
                        uint32_t *h_layer_offsets /*[nlayers]*/);
int chr_bvh_result_free(chr_bvh_result *r);

/* ------------------------------------------------------------- flatten helper
 * replaces: the np.unique(rows, return_inverse=True) of Mesh.remove_duplicate_vertices
 * (chroma/geometry.py:71-81, called by Geometry.flatten, geometry.py:337-391)
 * where every set of equal rows is bit-identical (so which duplicate numpy
 * keeps cannot matter): rows sorted lexicographically by float value (x, then
 * y, then z; -0.0 == +0.0), duplicates merged.  out_vertices (>= n rows)
 * receives the unique rows, *nunique their count, inverse[i] the unique row of
 * input row i.  Returns CHR_ERR_INVALID for a NaN, or a set of equal rows that
 * mixes +0.0 and -0.0 (the caller then uses numpy). */
int chr_unique_vertices(const float *h_vertices, uint64_t n, float *h_out_vertices, uint64_t *nunique,
                        int64_t *h_inverse);

/* ------------------------------------------------------------- traversal BVH
 * The layout the gfx950 walk uses (csrc/wide_bvh.h): an 8-wide SAH tree over
 * the reference BVH's own leaf boxes, each triangle carrying its reference DFS
 * rank.  chr_geometry_create builds it internally; these entries expose the
 * same host build for inspection and tests (no reference counterpart: it is
 * a derived acceleration structure, not part of the reference's data).
 * Nodes are 96 bytes, triangle records 64 bytes (see wide_bvh.h). */
typedef struct chr_wide_result chr_wide_result;
int chr_wide_bvh_build(const chr_geometry_desc *desc, chr_wide_result **out);
int chr_wide_bvh_info(const chr_wide_result *r, uint32_t *nnodes, uint32_t *ntri,
                      uint32_t *max_depth, int32_t *usable);
int chr_wide_bvh_copy(const chr_wide_result *r, void *h_nodes /*[nnodes*96 B]*/,
                      void *h_tri /*[ntri*64 B]*/);
int chr_wide_bvh_free(chr_wide_result *r);

/* The traversal BVH in its compact, cacheable form.  The reference caches the
 * BVH its kernel walks, keyed by mesh MD5 (chroma/cache.py:209-236, used by
 * chroma/loader.py:131-160); here the structure the kernel walks is the wide
 * BVH, a function of the mesh and the reference BVH only.  Its compact form
 * keeps what the build decides -- the nodes, each triangle record's triangle
 * id and reference DFS rank -- and drops what the upload
 * derives from the geometry descriptor (vertices, reference leaf words,
 * material codes), so a cached copy cannot go stale against the materials. */
typedef struct chr_wide_bvh_desc {
    uint32_t nnodes;                /* 96-byte nodes (wide_bvh.h WideNode) */
    uint32_t nrec;                  /* triangle records = triangles reachable in the reference BVH */
    uint32_t max_depth;             /* levels below the root */
    int32_t usable;                 /* 0: the wide walk cannot be used (the exact-order walk is) */
    uint32_t leaf_max;              /* builder setting it was built with */
    const void *h_nodes;            /* [nnodes*96 B] */
    const uint32_t *h_rec_id;       /* [nrec] triangle id of record i */
    const uint32_t *h_rec_rank;     /* [nrec] its reference DFS rank (a permutation of [0, nrec)) */
} chr_wide_bvh_desc;
/* sizes and settings of a built result (pointers left NULL) */
int chr_wide_bvh_describe(const chr_wide_result *r, chr_wide_bvh_desc *out);
/* copy the compact form into caller arrays sized by chr_wide_bvh_describe */
int chr_wide_bvh_export(const chr_wide_result *r, void *h_nodes, uint32_t *h_rec_id, uint32_t *h_rec_rank);
/* the builder's settings as a short string ("w<format>-l<leaf max>"):
 * part of a cache key -- a compact form is reused only under the same settings */
int chr_wide_bvh_key(char *out, uint32_t n);
/* check a compact form against a geometry (every index in range, the ranks a
 * permutation, the depth within the walk's stack) and rebuild its 64-byte
 * triangle records [first, first+n) on the host (tests; the upload does the same) */
int chr_wide_bvh_records(const chr_geometry_desc *desc, const chr_wide_bvh_desc *wide, uint32_t first,
                         uint32_t n, void *h_tri /*[n*64 B]*/);
/* chr_geometry_create with a prebuilt (e.g. cached) traversal BVH instead of
 * building it: the same device layout and results, without the build.  The
 * compact form is validated first (CHR_ERR_INVALID if it does not fit desc);
 * one marked unusable selects the exact-order walk, as the build would. */
int chr_geometry_create_wide(const chr_geometry_desc *desc, const chr_wide_bvh_desc *wide,
                             chr_geometry **out);

/* Threads of the library's host-side parallel regions (BVH builds, record
 * fill, vertex merge).  Default: the usable cores (affinity mask capped by the
 * cgroup CPU quota) divided by $LOCAL_WORLD_SIZE; n = 0 restores the default.
 * No reference counterpart (the reference builds on the GPU). */
int chr_set_host_threads(int32_t n);
int32_t chr_get_host_threads(void);

/* ------------------------------------------------------------------- DAQ
 * replaces: chroma/cuda/daq.cu + GPUDaq (chroma/gpu/daq.py:37-101) and the
 * Detector struct (chroma/cuda/detector.h:4-22, uploaded by
 * chroma/gpu/detector.py:21-40).  Per-channel accumulators are u32 arrays of
 * ndaq*nchannels (copy i of channel c at i*stride + c): earliest time as the
 * float's bit pattern under unsigned atomicMin (daq.cu:5-10 keeps
 * float_to_sortable_int as a plain bit cast), charge as round(q/charge_unit)
 * under atomicAdd, history under atomicOr -- all order-independent, so the
 * result does not depend on the schedule. */
typedef struct chr_daq_detector {
    const int32_t *d_solid_id_to_channel_index;   /* [nsolids] */
    const float *d_time_cdf_x, *d_time_cdf_y;     /* [time_cdf_len] */
    const float *d_charge_cdf_x, *d_charge_cdf_y; /* [charge_cdf_len] */
    int32_t nchannels, time_cdf_len, charge_cdf_len;
    float charge_unit;                            /* charge_cdf_x[-1] / 2^16 (gpu/detector.py:39) */
} chr_daq_detector;

/* replaces: GPUDaq.begin_acquire (daq.py:56-60): time words = bits(maxtime), q and history = 0 */
int chr_daq_begin(uint32_t *d_time_int, uint32_t *d_q_int, uint32_t *d_history, uint32_t n, float maxtime,
                  void *stream);
/* replaces: GPUDaq.acquire (daq.py:62-91): run_daq (ndaq == 1, daq.cu:35-83) or
 * run_daq_many (ndaq > 1, daq.cu:85-145) over photons [start, start+n) with the
 * reference's chunking (slot = position in chunk; nthreads_per_block*max_blocks
 * slots for ndaq == 1, one photon per block of nthreads_per_block slots for
 * ndaq > 1).  d_normal_cache (2 words per slot, zero after chr_init_rng) holds
 * curand_normal's cached value; required only for ndaq > 1.  Synchronous. */
int chr_daq_acquire(const chr_photons *ph, uint32_t *d_rng_states, uint32_t rng_nslots, uint32_t *d_normal_cache,
                    uint32_t detection_state, int32_t start_photon, int32_t nphotons,
                    const uint32_t *d_solid_map, const chr_daq_detector *det,
                    uint32_t *d_time_int, uint32_t *d_q_int, uint32_t *d_history,
                    int32_t ndaq, int32_t stride, float global_weight,
                    int32_t nthreads_per_block, int32_t max_blocks, void *stream);
/* replaces: GPUDaq.end_acquire (daq.py:93-101): convert_sortable_int_to_float
 * over all n words, convert_charge_int_to_float over the first nchannels words
 * only (daq.cu:158-172; later DAQ copies keep charge 0, as in the reference). */
int chr_daq_end(const uint32_t *d_time_int, float *d_time, const uint32_t *d_q_int, float *d_q, uint32_t n,
                int32_t nchannels, float charge_unit, void *stream);

/* Detected photons per channel, ACCUMULATED into d_counts[nchannels] (u32; the
 * caller zeroes it): the selection of count_photon_hits (propagate.cu:172-199)
 * histogrammed by channel.  No reference counterpart -- it is the per-rank
 * array a photon-sharded run reduces over RCCL (chroma/gpu/shard.py). Async. */
int chr_channel_hit_counts(const chr_photons *ph, int32_t start_photon, int32_t nphotons,
                           uint32_t detection_state, const uint32_t *d_solid_map,
                           const int32_t *d_solid_id_to_channel_index, uint32_t *d_counts,
                           int32_t nchannels, void *stream);

/* ------------------------------------------------------------------- PDF
 * replaces: chroma/cuda/pdf.cu, launched by GPUPDF / GPUKernelPDF
 * (chroma/gpu/pdf.py:7-372).  Inputs are GPUChannels words (t, q: f32; DAQ
 * copy i of channel c at i*nchannels + c).  One work-item per channel, the
 * reference's accumulation order and float accumulators.  All async. */

/* replaces: bin_hits (pdf.cu:9-32; GPUPDF.add_hits_to_pdf, pdf.py:206-222).
 * d_pdf is [nchannels][tbins][qbins] u32.  Bins are clamped to the channel's
 * last bin (the reference can spill t == tmax-ulp into the next row). */
int chr_pdf_bin_hits(int32_t nchannels, const float *d_channel_q, const float *d_channel_time,
                     uint32_t *d_hitcount, int32_t tbins, float tmin, float tmax, int32_t qbins, float qmin,
                     float qmax, uint32_t *d_pdf, void *stream);
/* replaces: accumulate_bincount (pdf.cu:34-96; GPUPDF.accumulate_pdf_eval,
 * pdf.py:296-316).  d_work_queues: nhit*(ndaq+1) u32, word 0 of each queue
 * = 1 + queued entries (the caller fills 1). */
int chr_pdf_accumulate_bincount(int32_t nchannels, int32_t ndaq, const uint32_t *d_event_hit,
                                const float *d_event_time, const float *d_mc_time, uint32_t *d_hitcount,
                                uint32_t *d_bincount, float min_twidth, float tmin, float tmax,
                                int32_t min_bin_content, const uint32_t *d_map_channel_to_hit,
                                uint32_t *d_work_queues, void *stream);
/* replaces: accumulate_nearest_neighbor_block (pdf.cu:152-219; pdf.py:318-328):
 * per hit, the min_bin_content smallest of (stored table + queued distances),
 * ascending.  min_bin_content <= 8192 (the reference's table holds 1000). */
int chr_pdf_accumulate_nearest(int32_t nhit, int32_t ndaq, const uint32_t *d_map_hit_to_channel,
                               const uint32_t *d_work_queues, const float *d_event_time,
                               const float *d_mc_time, float *d_nearest_mc, int32_t min_bin_content,
                               void *stream);
/* replaces: accumulate_moments (pdf.cu:223-266; GPUKernelPDF.accumulate_moments, pdf.py:42-59) */
int chr_pdf_accumulate_moments(int32_t time_only, int32_t nchannels, const float *d_mc_time,
                               const float *d_mc_charge, float tmin, float tmax, float qmin, float qmax,
                               uint32_t *d_mom0, float *d_t_mom1, float *d_t_mom2, float *d_q_mom1,
                               float *d_q_mom2, void *stream);
/* replaces: accumulate_kernel_eval (pdf.cu:271-368; GPUKernelPDF.accumulate_kernel, pdf.py:139-158) */
int chr_pdf_accumulate_kernel_eval(int32_t time_only, int32_t nchannels, const uint32_t *d_event_hit,
                                   const float *d_event_time, const float *d_event_charge,
                                   const float *d_mc_time, const float *d_mc_charge, float tmin, float tmax,
                                   float qmin, float qmax, const float *d_inv_time_bw,
                                   const float *d_inv_charge_bw, uint32_t *d_hitcount, float *d_time_pdf,
                                   float *d_charge_pdf, void *stream);

/* ---------------------------------------------------------------- renderer
 * replaces: the `render` kernel (chroma/cuda/render.cu:37-183) as launched by
 * GPURays.render (chroma/gpu/render.py:47-62).  Rays float3-packed [n*3] (not
 * normalised, as the reference); d_colors: one ARGB word per triangle
 * (reference GPUGeometry.colors); per ray: d_dx / d_color (float4) hold
 * alpha_depth entries, d_dxlen the entries kept (0 = start afresh; a
 * non-zero count merges this render into the previous one, keep_last_render).
 * d_pixels[i] = composited ARGB or bg_color. */
int chr_render(const chr_geometry *g, uint32_t nrays, const float *d_pos, const float *d_dir,
               const uint32_t *d_colors, uint32_t alpha_depth, uint32_t *d_pixels, float *d_dx,
               uint32_t *d_dxlen, float *d_color, uint32_t bg_color, void *stream);
/* replaces: transform.cu:9-48 (translate / rotate / rotate_around_point of float3 arrays,
 * GPURays.translate/rotate/rotate_around_point, gpu/render.py:30-45) */
int chr_transform_translate(uint32_t n, float *d_a, float vx, float vy, float vz, void *stream);
int chr_transform_rotate(uint32_t n, float *d_a, float phi, float ax, float ay, float az, void *stream);
int chr_transform_rotate_around_point(uint32_t n, float *d_a, float phi, float ax, float ay, float az,
                                      float px, float py, float pz, void *stream);
/* replaces: hybrid_render.cu:61-131 update_xyz_lookup (camera.py:246-258): work-item k
 * (k < nthreads, triangle id = k + offset < total_threads, RNG slot k) shoots light from
 * position[3] at a random point of its triangle; if that triangle is the first hit, the
 * photon is propagated to its first diffuse reflection and cos_theta * xyz[3] is added to
 * the reflecting triangle's float3 entry of d_lookup1 (inside-to-outside) or d_lookup2.
 * d_vertices / d_triangles: the mesh (float3 / uint3 packed). */
int chr_hybrid_update_xyz_lookup(const chr_geometry *g, const float *d_vertices, const uint32_t *d_triangles,
                                 int32_t nthreads, int32_t total_threads, int32_t offset, const float *position,
                                 uint32_t *d_rng_states, uint32_t rng_nslots, float wavelength, const float *xyz,
                                 float *d_lookup1, float *d_lookup2, int32_t max_steps, void *stream);
/* replaces: hybrid_render.cu:133-166 update_xyz_image (camera.py:260-275) */
int chr_hybrid_update_xyz_image(const chr_geometry *g, int32_t nthreads, uint32_t *d_rng_states,
                                uint32_t rng_nslots, const float *d_positions, const float *d_directions,
                                float wavelength, const float *xyz, const float *d_lookup1,
                                const float *d_lookup2, float *d_image, int32_t nlookup_calls,
                                int32_t max_steps, void *stream);
/* replaces: hybrid_render.cu:168-200 process_image (camera.py:277-282) */
int chr_hybrid_process_image(int32_t nthreads, const float *d_image, uint32_t *d_pixels, int32_t nimages,
                             void *stream);

/* ------------------------------------------------------------ self tests
 * The reference's unit-test kernels, run over this build's device math (the
 * functions the propagate kernels inline).  Tests only. */
enum chr_linalg_op {   /* replaces: the 20 kernels of test/linalg_test.cu, in order */
    CHR_LINALG_FLOAT3ADD = 0, CHR_LINALG_FLOAT3ADDEQUAL, CHR_LINALG_FLOAT3SUB, CHR_LINALG_FLOAT3SUBEQUAL,
    CHR_LINALG_FLOAT3ADDFLOAT, CHR_LINALG_FLOAT3ADDFLOATEQUAL, CHR_LINALG_FLOATADDFLOAT3, CHR_LINALG_FLOAT3SUBFLOAT,
    CHR_LINALG_FLOAT3SUBFLOATEQUAL, CHR_LINALG_FLOATSUBFLOAT3, CHR_LINALG_FLOAT3MULFLOAT,
    CHR_LINALG_FLOAT3MULFLOATEQUAL, CHR_LINALG_FLOATMULFLOAT3, CHR_LINALG_FLOAT3DIVFLOAT,
    CHR_LINALG_FLOAT3DIVFLOATEQUAL, CHR_LINALG_FLOATDIVFLOAT3, CHR_LINALG_DOT, CHR_LINALG_CROSS, CHR_LINALG_NORM,
    CHR_LINALG_MINUSFLOAT3, CHR_LINALG_NOPS
};
/* d_a, d_b: float3-packed [n*3]; d_out [n*3] (or [n] for DOT/NORM) */
int chr_selftest_linalg(int32_t op, uint32_t n, const float *d_a, const float *d_b, float c, float *d_out,
                        void *stream);
/* replaces: test/rotate_test.cu (rotate.h:21-28): d_out[i] = rotate(a[i], phi[i], n) */
int chr_selftest_rotate(uint32_t n, const float *d_a, const float *d_phi, float nx, float ny, float nz,
                        float *d_out, void *stream);
/* replaces: test/test_sample_cdf.cu (random.h:27-55): one draw per slot i < n from
 * RNG slot state i (SoA, chr_init_rng layout; states are not written back);
 * uniform_grid = 0: sample_cdf(cdf_x, cdf_y), 1: sample_cdf(x0, delta, cdf_y),
 * 2: the bucket-indexed form of 1 the propagate kernels use for re-emission time
 * CDFs (index built as chr_geometry_create builds it; synchronous) */
int chr_selftest_sample_cdf(uint32_t n, const uint32_t *d_states, uint32_t nslots, int32_t ncdf,
                            const float *d_cdf_x, const float *d_cdf_y, float x0, float delta,
                            int32_t uniform_grid, float *d_out, void *stream);

/* ------------------------------------------------------------- device profile
 * replaces: the CHROMA_DEVICE_PROFILE build (chroma/cuda/profile.h:9-37) and
 * chroma.gpu.profiler.device_fetch / device_reset / device_report
 * (chroma/gpu/profiler.py:207-288).  Region counters (calls, cycles) of the split
 * step kernels, compiled only into libchroma_amd_prof.so (-DCHR_DEVICE_PROFILE=1;
 * chroma.gpu._native loads it when $CHROMA_DEVICE_PROFILE is set).  cycles are
 * lane-cycles of the shader clock (s_memtime): per work-item, the wave's time spent in
 * the region while that work-item took part, summed over work-items -- the reference's
 * per-thread clock64 sums.  Regions 0-5 keep the reference's ids. */
enum {
    CHR_PROF_INTERSECT_MESH = 0,      /* trace_kernel walks: calls = walks, cycles = node + triangle steps */
    CHR_PROF_INTERSECT_NODE = 1,      /* trace_kernel node steps (8-child slab test + stack) */
    CHR_PROF_INTERSECT_TRIANGLE = 2,  /* trace_kernel triangle steps (incl. the reference leaf-box check) */
    CHR_PROF_INTERSECT_BOX = 3,       /* child boxes slab-tested (calls only: part of the node steps) */
    CHR_PROF_FILL_MATERIAL = 4,       /* shade_kernel finish_fill (normal, material, surface of the hit) */
    CHR_PROF_FILL_ANALYTIC = 5,       /* kept for the reference's id (no analytic solids here: 0) */
    CHR_PROF_TRACE_REFILL = 6,        /* trace_kernel: publishing results + fetching the next rays */
    CHR_PROF_TRACE_IDLE = 7,          /* trace_kernel: lanes without work while their wave steps */
    CHR_PROF_SHADE_PHYSICS = 8,       /* shade_kernel propagate_to_boundary / _at_surface / _at_boundary */
    CHR_PROF_SHADE_OTHER = 9,         /* shade_kernel: state fetch wait, write-back, masks */
    CHR_PROF_TAIL_WALK = 10,          /* propagate_tail_kernel: the wave-spread walks (calls = walks) */
    CHR_PROF_TAIL_PHYSICS = 11,       /* propagate_tail_kernel: finish_fill + physics of the steps */
    CHR_PROF_TAIL_OTHER = 12,         /* propagate_tail_kernel: photon load / write-back / waiting */
    CHR_PROF_TRACE_KERNEL = 13,       /* whole trace_kernel (calls = work-items) */
    CHR_PROF_SHADE_KERNEL = 14,       /* whole shade_kernel */
    CHR_PROF_TAIL_KERNEL = 15,        /* whole propagate_tail_kernel */
    CHR_PROF_TRACE_DRAIN = 16,        /* trace_kernel: a wave's last <= 8 walks, whole-wave (calls = walks) */
    /* the lone walker's wave-cycles per phase of its iterations (walk_lone, the default, has no
       separate fetch phase: its node / record loads are waited for inside EXPAND / TRIS): */
    CHR_PROF_LONE_REFILL = 17,        /* cursors refilled from the shared stack */
    CHR_PROF_LONE_FETCH = 18,         /* nodes + triangles loaded (issued and waited for) */
    CHR_PROF_LONE_EXPAND = 19,        /* children slab-tested, near child, pushes, triangle list */
    CHR_PROF_LONE_TRIS = 20,          /* triangles tested, nearest hit reduced */
    CHR_PROF_LONE_WALK = 21,          /* all of the above (calls = iterations) */
    /* a long-lived photon's tail steps (its steps beyond the 64th), wave cycles per phase: */
    CHR_PROF_LONG_WALK = 22,          /* the walk (calls = such steps) */
    CHR_PROF_LONG_FILL = 23,          /* finish_fill: the hit's record, normal, material, surface */
    CHR_PROF_LONG_TO_BOUNDARY = 24,   /* propagate_to_boundary */
    CHR_PROF_LONG_AT_BOUNDARY = 25,   /* propagate_at_surface / _at_boundary */
    CHR_PROF_LONG_OTHER = 26,         /* the rest of the step: the kernel's loop, ballots, the walk's set-up */
    CHR_PROF_NREGIONS = 27,
    CHR_PROF_COUNT = 64               /* counter array length (profile.h:16) */
};
/* 1 when this library was built with the device profile, else 0 */
int chr_device_profile_enabled(void);
/* zero the counters (replaces the chroma_prof_reset kernel); CHR_ERR_INVALID without the profile build */
int chr_device_profile_reset(void *stream);
/* copy n <= CHR_PROF_COUNT counters to host arrays and the shader clock (kHz) the
 * cycles convert with (hipDeviceAttributeClockRate); synchronises the device */
int chr_device_profile_fetch(uint64_t *h_calls, uint64_t *h_cycles, int32_t n, uint32_t *clock_khz);
/* Photon watch (diagnostics, profile build only; no reference counterpart):
 * every step of photon `photon` (its index in a batch's arrays; d_pos_array =
 * that batch's pos array, NULL: any batch) run by the shade or tail kernels is
 * recorded as 20 words -- kind (1 shade, 2 tail), queue position, hit triangle,
 * walk distance, pos in (3), dir in (3), last hit in, material1, absorption and
 * scattering lengths, pos out (3), history out, time out, RNG slot (the layout
 * of the oracle's orc_set_watch).  chr_watch_set clears the record count;
 * chr_watch_fetch copies min(count, max_records, 4096) records and the count. */
int chr_watch_set(uint32_t photon, const float *d_pos_array);
int chr_watch_fetch(uint32_t *h_out, uint32_t max_records, uint32_t *nrecords);
/* The walk of one ray by trace_kernel (profile build): h_origin non-NULL arms the
 * log for the ray with exactly this origin (3 floats); with h_origin NULL,
 * copies min(count, max_events, 8192) 8-word events (kind 1 start, 2 pop,
 * 3 node expansion, 4 triangle fetched, 5 triangle hit, 6 leaf-box check,
 * 7 drain, 8 drain publish, 9 publish) and the count. */
int chr_watch_ray(const float *h_origin, uint32_t *h_events, uint32_t max_events, uint32_t *nevents);

/* ------------------------------------------------------------- misc */
const char *chr_last_error(void);
int chr_version(void);
/* sha256 (16 hex) of the sources this library was built from (tools/source_sha.py:
 * csrc/ and include/), compiled in by the Makefile; bench.py compares it with the
 * tree's own (so_source_sha vs kernel_source_sha) */
const char *chr_source_sha(void);

#ifdef __cplusplus
}
#endif
#endif /* CHROMA_AMD_H */
