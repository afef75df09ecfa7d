"""STL mesh reader (drop-in for reference chroma/stl.py): ascii or binary,
optionally bz2-compressed; identical vertices are shared in first-seen order."""
import bz2
import struct

import numpy as np

from chroma.geometry import Mesh


def _open(filename, mode='rb'):
    return bz2.BZ2File(filename) if filename.endswith('.bz2') else open(filename, mode)


def _indexer():
    vertices, lookup = [], {}

    def index(v):
        if v not in lookup:
            lookup[v] = len(vertices)
            vertices.append(v)
        return lookup[v]
    return vertices, index


def mesh_from_ascii_stl(filename):
    vertices, index = _indexer()
    triangles, tri = [], []
    with _open(filename) as f:
        for raw in f:
            line = raw.decode('ascii').strip()
            if line.startswith('vertex'):
                tri.append(index(tuple(float(s) for s in line.split()[1:])))
                if len(tri) == 3:
                    triangles.append(tri)
                    tri = []
    return Mesh(np.array(vertices), np.array(triangles, dtype=np.uint32))


def mesh_from_binary_stl(filename):
    vertices, index = _indexer()
    triangles = []
    with _open(filename) as f:
        f.read(80)
        n = struct.unpack('<I', f.read(4))[0]
        for _ in range(n):
            rec = struct.unpack('<12fH', f.read(50))
            triangles.append([index(tuple(rec[3 + 3 * j:6 + 3 * j])) for j in range(3)])
    return Mesh(np.array(vertices), np.array(triangles, dtype=np.uint32))


def mesh_from_stl(filename):
    with _open(filename) as f:
        head = f.read(200)
    try:
        head.decode('ascii')
        return mesh_from_ascii_stl(filename)
    except (UnicodeDecodeError, ValueError, IndexError):
        return mesh_from_binary_stl(filename)
