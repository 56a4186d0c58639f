#!/bin/bash
# Register / scratch / LDS use of the kernels of one object of libcdbmerge (gfx950 code object).
# Usage: bash scripts/kres.sh engine.hip [regex]
set -e
OBJ=constdb_amd/build/obj/$1.o
D=$(mktemp -d)
objcopy -O binary --only-section=.hip_fatbin "$OBJ" $D/fat.bin
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$D/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$D/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $D/k.co > $D/notes.txt
python3 - "$D/notes.txt" "${2:-.}" <<'PY'
import re, sys
cur, out = {}, []
for line in open(sys.argv[1]):
    s = line.strip()
    if s.startswith('- .agpr_count') or s.startswith('- .args'):
        if cur: out.append(cur)
        cur = {}
    for k in ('.name:', '.private_segment_fixed_size:', '.vgpr_count:', '.sgpr_spill_count:', '.vgpr_spill_count:',
              '.group_segment_fixed_size:'):
        if s.startswith(k): cur[k] = s.split(':', 1)[1].strip()
if cur: out.append(cur)
for c in out:
    n = c.get('.name:', '?')
    if re.search(sys.argv[2], n):
        print(f"{n[:72]:72s} scratch {c.get('.private_segment_fixed_size:')} vgpr {c.get('.vgpr_count:')} "
              f"vspill {c.get('.vgpr_spill_count:')} sspill {c.get('.sgpr_spill_count:')} lds {c.get('.group_segment_fixed_size:')}")
PY
rm -rf $D
