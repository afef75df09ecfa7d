#!/usr/bin/env python3
"""Instruction mix of the kernels in a device assembly file (make asm):
usage: tools/isa_count.py chroma-lite_amd/csrc/_build/propagate.s [name-substring]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
want = sys.argv[2] if len(sys.argv) > 2 else 'trace_kernel'
for m in re.finditer(r'^(_Z\S+):\s*;\s*@', s, re.M):
    name = m.group(1)
    if want not in name:
        continue
    j = s.find('.Lfunc_end', m.end())
    body = s[m.end():j]
    ins = [ln.strip().split()[0] for ln in body.split('\n')
           if ln.startswith('\t') and ln.strip() and not ln.strip().startswith(('.', ';'))]
    c = Counter(ins)
    print(name, 'instructions', len(ins))
    for k in ('v_pk_fma_f32', 'v_fma_f32', 'v_pk_mul_f32', 'v_pk_add_f32', 'v_min3_f32', 'v_max3_f32',
              'v_cvt_f32_ubyte0', 'v_cvt_f32_ubyte1', 'v_cvt_f32_ubyte2', 'v_cvt_f32_ubyte3', 'v_cndmask_b32',
              'global_load_dwordx4', 's_waitcnt', 'ds_write_b32', 'ds_read_b32'):
        print('  %-22s %d' % (k, c[k]))
