"""ctypes binding of the C ABI in include/chroma_amd.h (libchroma_amd.so).

This is the only place Python touches native code.  The library is built
in-tree (chroma-lite_amd/csrc/Makefile -> chroma/_lib/libchroma_amd.so) and is
REQUIRED: there is no Python or CPU fallback for the GPU path, so a missing
library raises immediately.
"""
import ctypes
import os

_LIBDIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), '_lib')
# CHROMA_DEVICE_PROFILE=1: the build with the device region counters compiled in
# (the reference's -DCHROMA_DEVICE_PROFILE=1 kernels, profile.h; chroma.gpu.profiler.device_*)
DEVICE_PROFILE = os.environ.get('CHROMA_DEVICE_PROFILE', '').strip().lower() in ('1', 'true', 'yes', 'on')
_LIBPATH = os.path.join(_LIBDIR, 'libchroma_amd_prof.so' if DEVICE_PROFILE else 'libchroma_amd.so')
# dev A/B of alternative builds (still in-tree): CHROMA_AMD_LIB=/path/to/libchroma_amd*.so
_LIBPATH = os.environ.get('CHROMA_AMD_LIB', _LIBPATH)

c_u32 = ctypes.c_uint32
c_i32 = ctypes.c_int32
c_u64 = ctypes.c_uint64
c_f32 = ctypes.c_float
c_vp = ctypes.c_void_p
P_f32 = ctypes.POINTER(ctypes.c_float)
P_u32 = ctypes.POINTER(ctypes.c_uint32)


class MaterialDesc(ctypes.Structure):
    _fields_ = [('num_comp', c_u32), ('refractive_index', c_vp), ('absorption_length', c_vp),
                ('scattering_length', c_vp), ('comp_reemission_prob', c_vp),
                ('comp_reemission_wvl_cdf', c_vp), ('comp_reemission_time_cdf', c_vp),
                ('comp_absorption_length', c_vp)]


class SurfaceDesc(ctypes.Structure):
    _fields_ = [('present', c_i32), ('model', c_u32), ('transmissive', c_u32), ('thickness', c_f32),
                ('detect', c_vp), ('absorb', c_vp), ('reemit', c_vp), ('reflect_diffuse', c_vp),
                ('reflect_specular', c_vp), ('eta', c_vp), ('k', c_vp), ('reemission_cdf', c_vp),
                ('dichroic_nangles', c_u32), ('dichroic_angles', c_vp), ('dichroic_reflect', c_vp),
                ('dichroic_transmit', c_vp), ('angular_nangles', c_u32), ('angular_angles', c_vp),
                ('angular_transmit', c_vp), ('angular_reflect_specular', c_vp),
                ('angular_reflect_diffuse', c_vp)]


class WirePlaneDesc(ctypes.Structure):
    _fields_ = [('origin', c_f32 * 3), ('u', c_f32 * 3), ('v', c_f32 * 3), ('pitch', c_f32),
                ('radius', c_f32), ('umin', c_f32), ('umax', c_f32), ('vmin', c_f32), ('vmax', c_f32),
                ('v0', c_f32), ('surface_index', c_i32), ('material_outer_index', c_i32),
                ('material_inner_index', c_i32), ('color', c_u32)]


class GeometryDesc(ctypes.Structure):
    _fields_ = [('nvertices', c_u32), ('ntriangles', c_u32), ('nnodes', c_u32), ('nmaterials', c_u32),
                ('nsurfaces', c_u32), ('nwireplanes', c_u32), ('h_vertices', c_vp), ('h_triangles', c_vp),
                ('h_material_codes', c_vp), ('h_nodes', c_vp), ('world_origin', c_f32 * 3),
                ('world_scale', c_f32), ('wavelength_n', c_u32), ('wavelength_start', c_f32),
                ('wavelength_step', c_f32), ('time_n', c_u32), ('time_start', c_f32), ('time_step', c_f32),
                ('materials', ctypes.POINTER(MaterialDesc)), ('surfaces', ctypes.POINTER(SurfaceDesc)),
                ('wireplanes', ctypes.POINTER(WirePlaneDesc))]


class WideBvhDesc(ctypes.Structure):
    """chr_wide_bvh_desc: the traversal BVH in compact (cacheable) form."""
    _fields_ = [('nnodes', c_u32), ('nrec', c_u32), ('max_depth', c_u32), ('usable', c_i32),
                ('leaf_max', c_u32), ('h_nodes', c_vp), ('h_rec_id', c_vp), ('h_rec_rank', c_vp)]


class PhotonsDesc(ctypes.Structure):
    _fields_ = [('d_pos', c_vp), ('d_dir', c_vp), ('d_pol', c_vp), ('d_wavelengths', c_vp), ('d_t', c_vp),
                ('d_weights', c_vp), ('d_flags', c_vp), ('d_last_hit_triangles', c_vp), ('d_evidx', c_vp)]


class PropagateStats(ctypes.Structure):
    _fields_ = [('steps_run', c_u32), ('launches', c_u32), ('final_alive', c_u32), ('stack_overflows', c_u32),
                ('kernel_ms', ctypes.c_double), ('nodes_visited', c_u64), ('triangles_tested', c_u64),
                ('traversals', c_u64), ('wave_node_steps', c_u64), ('wave_triangle_steps', c_u64),
                ('wave_fill_cycles', c_u64), ('wave_step_cycles', c_u64), ('trace_ms', ctypes.c_double),
                ('trace_launches', c_u32), ('reserved', c_u32), ('trace_rays', c_u64),
                ('trace_ms_n', c_u32), ('trace_launch_ms', c_f32 * 32), ('flat_walks', c_u32),
                ('flat_walks_whole', c_u32), ('tail_photons', c_u32), ('tail_ms', ctypes.c_double),
                ('tail_max_steps', c_u32), ('tail_slowest_steps', c_u32), ('tail_max_cycles', c_u64),
                ('tail_long_photons', c_u32), ('reserved2', c_u32), ('tail_long_steps', c_u64),
                ('tail_long_ticks', c_u64), ('tail_long_walk_ticks', c_u64), ('tail_long_walk_iterations', c_u64),
                ('host_syncs', c_u32), ('tail_long_paired_steps', c_u32), ('trace_launch_rays', c_u32 * 32)]


class KernelAttr(ctypes.Structure):
    _fields_ = [('private_bytes', c_u64), ('lds_bytes', c_u64), ('vgprs', ctypes.c_int32),
                ('max_threads', ctypes.c_int32), ('name', ctypes.c_char * 96)]


_SIGNATURES = {
    'chr_geometry_create': (c_i32, [ctypes.POINTER(GeometryDesc), ctypes.POINTER(c_vp)]),
    'chr_geometry_destroy': (c_i32, [c_vp]),
    'chr_geometry_device_bytes': (c_i32, [c_vp, ctypes.POINTER(c_u64)]),
    'chr_walk_lone_timing': (c_i32, [c_vp, c_vp, c_u32, c_u32, c_u32, c_i32, c_vp, c_vp]),
    'chr_geometry_phys_words': (c_i32, [c_vp, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    'chr_init_rng': (c_i32, [c_vp, c_u32, c_u64, c_u64, c_vp]),
    'chr_rng_download': (c_i32, [c_vp, c_u32, c_vp, c_vp]),
    'chr_propagate_scratch_words': (c_u64, [c_u32]),
    'chr_propagate_chunk': (c_i32, [c_vp, ctypes.POINTER(PhotonsDesc), c_vp, c_u32, c_i32, c_i32, c_vp, c_vp,
                                    c_i32, c_i32, c_i32, c_vp, c_vp]),
    'chr_propagate': (c_i32, [c_vp, ctypes.POINTER(PhotonsDesc), c_u32, c_u32, c_u32, c_vp, c_u32, c_i32, c_i32,
                              c_i32, c_i32, c_i32, ctypes.POINTER(PropagateStats), c_vp]),
    'chr_propagate_batches': (c_i32, [c_vp, ctypes.POINTER(PhotonsDesc), c_vp, c_vp, c_vp, c_u32, c_vp, c_u32, c_i32,
                                      c_i32, c_i32, c_i32, c_i32, ctypes.POINTER(PropagateStats), c_vp]),
    'chr_photon_hits': (c_i32, [ctypes.POINTER(PhotonsDesc), c_i32, c_i32, c_u32, c_vp, c_vp,
                                ctypes.POINTER(PhotonsDesc), c_vp, ctypes.POINTER(c_u32), c_vp]),
    'chr_select_photons': (c_i32, [ctypes.POINTER(PhotonsDesc), c_i32, c_i32, c_u32, ctypes.POINTER(PhotonsDesc),
                                   ctypes.POINTER(c_u32), c_vp]),
    'chr_copy_photon_queue': (c_i32, [ctypes.POINTER(PhotonsDesc), c_i32, c_i32, c_vp, ctypes.POINTER(PhotonsDesc),
                                      c_vp]),
    'chr_photon_duplicate': (c_i32, [ctypes.POINTER(PhotonsDesc), c_i32, c_i32, c_i32, c_i32, c_vp]),
    'chr_distance_to_mesh': (c_i32, [c_vp, c_u32, c_vp, c_vp, c_vp, c_vp]),
    'chr_kernel_info': (c_i32, [c_i32, ctypes.POINTER(KernelAttr)]),
    'chr_selftest_linalg': (c_i32, [c_i32, c_u32, c_vp, c_vp, c_f32, c_vp, c_vp]),
    'chr_selftest_rotate': (c_i32, [c_u32, c_vp, c_vp, c_f32, c_f32, c_f32, c_vp, c_vp]),
    'chr_selftest_sample_cdf': (c_i32, [c_u32, c_vp, c_u32, c_i32, c_vp, c_vp, c_f32, c_f32, c_i32, c_vp, c_vp]),
    'chr_unique_vertices': (c_i32, [c_vp, c_u64, c_vp, ctypes.POINTER(c_u64), c_vp]),
    'chr_bvh_build_grid': (c_i32, [c_vp, c_u32, c_vp, c_u32, c_i32, ctypes.POINTER(c_vp)]),
    'chr_bvh_result_info': (c_i32, [c_vp, ctypes.POINTER(c_u32), ctypes.POINTER(c_u32), c_vp,
                                    ctypes.POINTER(c_f32)]),
    'chr_bvh_result_copy': (c_i32, [c_vp, c_vp, c_vp]),
    'chr_bvh_result_free': (c_i32, [c_vp]),
    'chr_wide_bvh_build': (c_i32, [ctypes.POINTER(GeometryDesc), ctypes.POINTER(c_vp)]),
    'chr_wide_bvh_info': (c_i32, [c_vp, ctypes.POINTER(c_u32), ctypes.POINTER(c_u32), ctypes.POINTER(c_u32),
                                  ctypes.POINTER(ctypes.c_int32)]),
    'chr_wide_bvh_copy': (c_i32, [c_vp, c_vp, c_vp]),
    'chr_wide_bvh_free': (c_i32, [c_vp]),
    'chr_wide_bvh_describe': (c_i32, [c_vp, ctypes.POINTER(WideBvhDesc)]),
    'chr_wide_bvh_export': (c_i32, [c_vp, c_vp, c_vp, c_vp]),
    'chr_wide_bvh_key': (c_i32, [ctypes.c_char_p, c_u32]),
    'chr_wide_bvh_records': (c_i32, [ctypes.POINTER(GeometryDesc), ctypes.POINTER(WideBvhDesc), c_u32, c_u32, c_vp]),
    'chr_geometry_create_wide': (c_i32, [ctypes.POINTER(GeometryDesc), ctypes.POINTER(WideBvhDesc),
                                         ctypes.POINTER(c_vp)]),
    'chr_set_host_threads': (c_i32, [c_i32]),
    'chr_get_host_threads': (c_i32, []),
    'chr_daq_begin': (c_i32, [c_vp, c_vp, c_vp, c_u32, c_f32, c_vp]),
    'chr_daq_acquire': (c_i32, [ctypes.POINTER(PhotonsDesc), c_vp, c_u32, c_vp, c_u32, c_i32, c_i32, c_vp, c_vp,
                                c_vp, c_vp, c_vp, c_i32, c_i32, c_f32, c_i32, c_i32, c_vp]),
    'chr_daq_end': (c_i32, [c_vp, c_vp, c_vp, c_vp, c_u32, c_i32, c_f32, c_vp]),
    'chr_init_rng_subseq': (c_i32, [c_vp, c_u32, c_u64, c_u64, c_u64, c_vp]),
    'chr_channel_hit_counts': (c_i32, [ctypes.POINTER(PhotonsDesc), c_i32, c_i32, c_u32, c_vp, c_vp, c_vp, c_i32,
                                       c_vp]),
    'chr_pdf_bin_hits': (c_i32, [c_i32, c_vp, c_vp, c_vp, c_i32, c_f32, c_f32, c_i32, c_f32, c_f32, c_vp, c_vp]),
    'chr_pdf_accumulate_bincount': (c_i32, [c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_f32, c_i32,
                                            c_vp, c_vp, c_vp]),
    'chr_pdf_accumulate_nearest': (c_i32, [c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp]),
    'chr_pdf_accumulate_moments': (c_i32, [c_i32, c_i32, c_vp, c_vp, c_f32, c_f32, c_f32, c_f32, c_vp, c_vp, c_vp,
                                           c_vp, c_vp, c_vp]),
    'chr_pdf_accumulate_kernel_eval': (c_i32, [c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_f32, c_f32,
                                               c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    'chr_render': (c_i32, [c_vp, c_u32, c_vp, c_vp, c_vp, c_u32, c_vp, c_vp, c_vp, c_vp, c_u32, c_vp]),
    'chr_transform_translate': (c_i32, [c_u32, c_vp, c_f32, c_f32, c_f32, c_vp]),
    'chr_transform_rotate': (c_i32, [c_u32, c_vp, c_f32, c_f32, c_f32, c_f32, c_vp]),
    'chr_transform_rotate_around_point': (c_i32, [c_u32, c_vp, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32,
                                                  c_vp]),
    'chr_hybrid_update_xyz_lookup': (c_i32, [c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_u32, c_f32, c_vp,
                                             c_vp, c_vp, c_i32, c_vp]),
    'chr_hybrid_update_xyz_image': (c_i32, [c_vp, c_i32, c_vp, c_u32, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_vp,
                                            c_i32, c_i32, c_vp]),
    'chr_hybrid_process_image': (c_i32, [c_i32, c_vp, c_vp, c_i32, c_vp]),
    'chr_device_profile_enabled': (c_i32, []),
    'chr_device_profile_reset': (c_i32, [c_vp]),
    'chr_device_profile_fetch': (c_i32, [c_vp, c_vp, c_i32, ctypes.POINTER(c_u32)]),
    'chr_watch_set': (c_i32, [c_u32, c_vp]),
    'chr_watch_fetch': (c_i32, [c_vp, c_u32, ctypes.POINTER(c_u32)]),
    'chr_watch_ray': (c_i32, [c_vp, c_vp, c_u32, ctypes.POINTER(c_u32)]),
    'chr_last_error': (ctypes.c_char_p, []),
    'chr_version': (c_i32, []),
    'chr_source_sha': (ctypes.c_char_p, []),
}

EXPORTED = tuple(_SIGNATURES)

_lib = None


class NativeError(RuntimeError):
    """A nonzero chr_status from libchroma_amd (message = chr_last_error())."""


def library_path():
    return _LIBPATH


def lib():
    """Load libchroma_amd.so (once).  Raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIBPATH):
            raise ImportError('%s not found at %s: build it with `make -C chroma-lite_amd/csrc` '
                              '(or __graft_entry__.build())' % (os.path.basename(_LIBPATH), _LIBPATH))
        l = ctypes.CDLL(_LIBPATH)
        for name, (res, args) in _SIGNATURES.items():
            if 'CHROMA_AMD_LIB' in os.environ and not hasattr(l, name):
                continue     # dev A/B against an older build
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def check(rc, what=''):
    if rc != 0:
        msg = lib().chr_last_error().decode(errors='replace')
        raise NativeError('%s failed (status %d): %s' % (what, rc, msg))
    return rc


# chroma.gpu.profiler installs a timer here while host-side profiling is on
# (the reference wraps every PyCUDA kernel function, profiler.py:68-139; every
# launch here goes through call())
call_hook = None


def call(name, *args):
    if call_hook is not None:
        return call_hook(name, lambda: check(getattr(lib(), name)(*args), name))
    return check(getattr(lib(), name)(*args), name)


def kernel_info():
    """Code-object resources of the default propagate kernels (chr_kernel_info):
    list of dicts {name, private_bytes, lds_bytes, vgprs, max_threads}."""
    out = []
    for which in range(4):
        a = KernelAttr()
        call('chr_kernel_info', which, ctypes.byref(a))
        out.append(dict(name=a.name.decode(), private_bytes=int(a.private_bytes), lds_bytes=int(a.lds_bytes),
                        vgprs=int(a.vgprs), max_threads=int(a.max_threads)))
    return out


def set_host_threads(n):
    """Threads of the library's host-side parallel regions (chr_set_host_threads;
    0 restores the default: usable cores / $LOCAL_WORLD_SIZE)."""
    call('chr_set_host_threads', int(n))


def host_threads():
    return int(lib().chr_get_host_threads())
