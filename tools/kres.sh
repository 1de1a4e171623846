#!/bin/bash
# VGPR / spill / LDS of the Schur kernels in the built library (host-side check
# after a build; reads the gfx950 code object's metadata notes).
set -e
LIB=${1:-superlu_dist_amd/lib/libslu_mi355x.so}
PAT=${2:-schur_big}
T=$(mktemp -d)
objcopy -O binary --only-section=.hip_fatbin "$LIB" "$T/fat.bin"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$T/fat.bin" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/dev.o"
/opt/rocm/lib/llvm/bin/llvm-readobj --notes "$T/dev.o" > "$T/notes.txt"
python3 - "$T/notes.txt" "$PAT" <<'PY'
import re, sys
t = open(sys.argv[1]).read()
for blk in t.split('  - .agpr_count')[1:]:
    m = re.search(r'\.name:\s+(\S+)', blk)
    if not m or sys.argv[2] not in m.group(1):
        continue
    g = lambda k: (re.search(r'\.' + k + r':\s+(\S+)', blk) or [None, None])[1]
    print(f"{m.group(1)[:60]:60s} vgpr {g('vgpr_count')} spill {g('vgpr_spill_count')} lds {g('group_segment_fixed_size')}")
PY
rm -rf "$T"
