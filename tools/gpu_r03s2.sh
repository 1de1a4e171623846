#!/bin/bash
# Round 3: A/B of the swizzled unpadded LDS stages in k_schur_big (ablib/swz) and the k-stride lane mapping (ablib/kstr).
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_bench.sh ${1:-r03s2}_ab swz kstr
