#!/usr/bin/env python3
"""sha256 (16 hex) of the sources libchroma_amd.so is built from (csrc/*.hip,
*.h, *.cpp, the Makefile, include/*.h): the stamp that ties a committed PMC
record to the kernels it measured, and (compiled into the library by the
Makefile, chr_source_sha) a shipped .so to the tree it came from.

usage: tools/source_sha.py                 print the sha
       tools/source_sha.py --header FILE   write `#define CHR_SOURCE_SHA "<sha>"` to FILE
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_source_sha(root=ROOT):
    h = hashlib.sha256()
    csrc = os.path.join(root, 'chroma-lite_amd', 'csrc')
    inc = os.path.join(root, 'include')
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc)
                   if f.endswith(('.hip', '.h', '.cpp')) or f == 'Makefile')
    files += sorted(os.path.join(inc, f) for f in os.listdir(inc) if f.endswith('.h'))
    for p in files:
        h.update(os.path.relpath(p, root).encode())
        with open(p, 'rb') as f:
            h.update(f.read())
    return h.hexdigest()[:16]


if __name__ == '__main__':
    sha = kernel_source_sha()
    if len(sys.argv) == 3 and sys.argv[1] == '--header':
        with open(sys.argv[2], 'w') as f:
            f.write('#define CHR_SOURCE_SHA "%s"\n' % sha)
    else:
        print(sha)
