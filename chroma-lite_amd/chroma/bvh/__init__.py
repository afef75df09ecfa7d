"""Bounding volume hierarchy data model and builders (drop-in for reference
chroma/bvh/).  make_recursive_grid_bvh runs the host C++ builder in
libchroma_amd.so; no GPU is needed to build."""
from chroma.bvh.bvh import *  # noqa: F401,F403
from chroma.bvh.grid import make_recursive_grid_bvh  # noqa: F401
from chroma.bvh.simple import make_simple_bvh  # noqa: F401
