"""The traversal BVH the kernels walk, in its compact form, and its cache.

The reference caches the BVH its kernel walks, keyed by mesh MD5, so a run
does not rebuild it (chroma/cache.py:209-236 save_bvh / load_bvh, used by
chroma/loader.py:131-160).  Here the kernels walk the 8-wide gfx950 BVH that
libchroma_amd builds over the reference BVH (csrc/wide_bvh.cpp): 33-36 s of
host work for the 29k-PMT detector, which every process creating a
GPUGeometry would repeat.  Its compact form (chr_wide_bvh_desc: 96-byte
nodes, each triangle record's triangle id and reference DFS rank, the
nothing else) is a function of the mesh and the reference BVH alone; the
upload rebuilds the 64-byte triangle records from the geometry
(chr_geometry_create_wide), so a cached copy cannot go stale against the
materials.

Cache layout, next to the reference BVH it was built from:
``<cache_dir>/bvh/<mesh md5>/<bvh name>.wide/<builder key>/`` holding
``nodes.npy rec_id.npy rec_rank.npy meta.json`` (plain .npy files,
memory-mapped on load, read with allow_pickle=False).  ``meta.json`` records
a fingerprint of the reference BVH (a hash of its whole node array); a
mismatch means rebuild, and so do arrays of the wrong type or shape.
``$CHROMA_WIDE_CACHE=0`` turns the cache off.
"""
import ctypes
import hashlib
import json
import os
import time

import numpy as np

from chroma.gpu import _native
from chroma.log import logger

_ARRAYS = ('nodes', 'rec_id', 'rec_rank')


def builder_key():
    """The builder's settings as a cache key (chr_wide_bvh_key): a cached
    compact form is reused only under the same settings and format."""
    buf = ctypes.create_string_buffer(64)
    _native.call('chr_wide_bvh_key', buf, 64)
    return buf.value.decode()


def fingerprint(bvh):
    """The identity of a reference BVH: node count, world coordinates and a
    hash of every node (xxh3-128, ~0.3 s for the 29k detector's 3.8 GB of
    nodes; sha1 when xxhash is not importable).  A BVH rebuilt under the same
    name that differs in any node never reuses the traversal BVH built from
    the old one."""
    u = np.ascontiguousarray(bvh.nodes).view(np.uint32).reshape(-1, 4)
    try:
        import xxhash
        h, tag = xxhash.xxh3_128(), 'xxh3:'
    except ImportError:
        h, tag = hashlib.sha1(), 'sha1:'
    h.update(np.asarray([len(u)], np.int64).tobytes())
    h.update(np.asarray(bvh.world_coords.world_origin, np.float32).tobytes())
    h.update(np.asarray([bvh.world_coords.world_scale], np.float32).tobytes())
    if len(u):
        h.update(memoryview(u).cast('B'))
    return tag + h.hexdigest()


class WideBVH(object):
    """Compact traversal BVH: arrays + the facts chr_wide_bvh_desc carries."""

    def __init__(self, nodes, rec_id, rec_rank, max_depth, usable, leaf_max, key):
        self.nodes = nodes            # uint8 (nnodes, 96)
        self.rec_id = rec_id          # uint32 (nrec,)
        self.rec_rank = rec_rank      # uint32 (nrec,)
        self.max_depth, self.usable, self.leaf_max, self.key = int(max_depth), bool(usable), int(leaf_max), key

    def desc(self):
        ptr = lambda a: a.ctypes.data if a.size else None   # noqa: E731
        d = _native.WideBvhDesc()
        d.nnodes, d.nrec = len(self.nodes), len(self.rec_id)
        d.max_depth, d.usable, d.leaf_max = self.max_depth, int(self.usable), self.leaf_max
        d.h_nodes, d.h_rec_id, d.h_rec_rank = ptr(self.nodes), ptr(self.rec_id), ptr(self.rec_rank)
        return d

    def records(self, packed, first=0, n=None):
        """The 64-byte triangle records [first, first+n) as the upload rebuilds
        them (chr_wide_bvh_records), as uint8 (n, 64)."""
        n = len(self.rec_id) - first if n is None else n
        out = np.zeros((n, 64), np.uint8)
        _native.call('chr_wide_bvh_records', ctypes.byref(packed.desc()), ctypes.byref(self.desc()), first, n,
                     out.ctypes.data)
        return out


def build(packed):
    """Build the traversal BVH of a PackedGeometry on the host (chr_wide_bvh_build)
    and return its compact form."""
    h = ctypes.c_void_p()
    _native.call('chr_wide_bvh_build', ctypes.byref(packed.desc()), ctypes.byref(h))
    try:
        d = _native.WideBvhDesc()
        _native.call('chr_wide_bvh_describe', h, ctypes.byref(d))
        nodes = np.empty((d.nnodes, 96), np.uint8)
        rec_id = np.empty(d.nrec, np.uint32)
        rec_rank = np.empty(d.nrec, np.uint32)
        _native.call('chr_wide_bvh_export', h, nodes.ctypes.data, rec_id.ctypes.data, rec_rank.ctypes.data)
    finally:
        _native.lib().chr_wide_bvh_free(h)
    return WideBVH(nodes, rec_id, rec_rank, d.max_depth, d.usable, d.leaf_max, builder_key())


def cache_enabled():
    return os.environ.get('CHROMA_WIDE_CACHE', '1').strip().lower() not in ('0', 'false', 'no', 'off')


def directory(cache_dir, mesh_hash, name, key):
    return os.path.join(cache_dir, 'bvh', mesh_hash, '%s.wide' % name, key)


def save(wide, cache_dir, mesh_hash, name, fp):
    """Write the compact form next to its reference BVH; a unique temporary
    directory renamed into place, so concurrent writers never share files."""
    final = directory(cache_dir, mesh_hash, name, wide.key)
    parent = os.path.dirname(final)
    os.makedirs(parent, exist_ok=True)
    tmp = '%s.%d.tmp' % (final, os.getpid())
    os.makedirs(tmp, exist_ok=True)
    for a in _ARRAYS:
        np.save(os.path.join(tmp, a + '.npy'), np.ascontiguousarray(getattr(wide, a)), allow_pickle=False)
    with open(os.path.join(tmp, 'meta.json'), 'w') as f:
        json.dump({'fingerprint': fp, 'max_depth': wide.max_depth, 'usable': wide.usable,
                   'leaf_max': wide.leaf_max, 'key': wide.key}, f)
    import shutil
    for _ in range(2):
        try:
            os.rename(tmp, final)
            return
        except OSError:
            pass
        # an entry is there: another process's (keep it) or a stale or corrupt one (replace it)
        if load(cache_dir, mesh_hash, name, wide.key, fp) is not None:
            break
        shutil.rmtree(final, ignore_errors=True)
    shutil.rmtree(tmp, ignore_errors=True)


def load(cache_dir, mesh_hash, name, key, fp):
    """The cached compact form (arrays memory-mapped), or None when absent or
    built from another reference BVH."""
    d = directory(cache_dir, mesh_hash, name, key)
    try:
        with open(os.path.join(d, 'meta.json')) as f:
            meta = json.load(f)
    except (OSError, ValueError):
        return None
    if meta.get('fingerprint') != fp or meta.get('key') != key:
        return None
    try:
        arrs = {}
        for a in _ARRAYS:      # the large arrays memory-mapped (page cache, no heap copy)
            f = os.path.join(d, a + '.npy')
            arrs[a] = np.load(f, mmap_mode='r' if os.path.getsize(f) > (1 << 20) else None, allow_pickle=False)
    except (OSError, ValueError) as e:
        logger.warning('traversal BVH cache %s unreadable: %s', d, e)
        return None
    # the C side reads nnodes * 96 node bytes and nrec ids / ranks: arrays of another
    # type or shape are a corrupt entry, not something to hand it
    nodes, rid, rrank = arrs['nodes'], arrs['rec_id'], arrs['rec_rank']
    if (nodes.dtype != np.uint8 or nodes.ndim != 2 or nodes.shape[1] != 96 or rid.dtype != np.uint32 or
            rrank.dtype != np.uint32 or rid.ndim != 1 or rrank.shape != rid.shape):
        logger.warning('traversal BVH cache %s: arrays of the wrong type or shape (nodes %s %s, rec_id %s %s, '
                       'rec_rank %s %s): rebuilding', d, nodes.dtype, nodes.shape, rid.dtype, rid.shape,
                       rrank.dtype, rrank.shape)
        return None
    return WideBVH(arrs['nodes'], arrs['rec_id'], arrs['rec_rank'], meta['max_depth'], meta['usable'],
                   meta['leaf_max'], key)


def discard(bvh):
    """Forget a traversal BVH that failed validation on upload: the copy
    attached to the BVH and its cache entry (the next obtain() rebuilds)."""
    import shutil
    w = getattr(bvh, 'wide', None)
    bvh.wide = None
    ref = getattr(bvh, 'cache_ref', None)
    if ref and w is not None:
        shutil.rmtree(directory(ref[0], ref[1], ref[2], w.key), ignore_errors=True)


def obtain(bvh, packed, fresh=False):
    """(WideBVH, source) for a geometry's reference BVH: the copy attached to
    the BVH object ('memory'), its cache entry ('cache'), or a fresh host build
    ('built', then written to the cache when the BVH came from one; fresh=True
    always builds).  The BVH object carries ``cache_ref = (cache_dir, mesh_hash,
    name)`` when it was loaded from or saved to a chroma.cache.Cache."""
    key = builder_key()
    w = getattr(bvh, 'wide', None)
    if w is not None and w.key == key and not fresh:
        return w, 'memory'
    ref = getattr(bvh, 'cache_ref', None) if cache_enabled() else None
    fp = fingerprint(bvh) if ref else None
    if ref and not fresh:
        w = load(ref[0], ref[1], ref[2], key, fp)
        if w is not None:
            bvh.wide = w
            return w, 'cache'
    t0 = time.time()
    w = build(packed)
    logger.info('traversal BVH built in %.1fs (%d nodes, %d records)', time.time() - t0, len(w.nodes), len(w.rec_id))
    if ref:
        try:
            save(w, ref[0], ref[1], ref[2], fp)
            w2 = load(ref[0], ref[1], ref[2], key, fp)   # keep the file-backed copy, not 2 GB of heap
            w = w2 if w2 is not None else w
        except OSError as e:
            logger.warning('traversal BVH cache not written: %s', e)
    bvh.wide = w
    return w, 'built'


def prepare(geometry):
    """Make the traversal BVH of a geometry available (cache or build) without
    a GPU: e.g. rank 0 of a multi-GPU job before the other ranks load it."""
    from chroma.gpu.packing import PackedGeometry
    return obtain(geometry.bvh, PackedGeometry(geometry))[1]
