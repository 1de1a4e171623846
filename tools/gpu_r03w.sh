#!/bin/bash
# Round 3: the 100^3 drop-in with the per-call timing breakdown, then an A/B of
# the unclamped 16-byte B loads in k_schur_big (ablib/b16, -DSLU_SB_B16).
set -o pipefail
export TMPDIR=/tmp
bash tools/dropin_solve_n100.sh ${1:-r03w}_solve100 && bash tools/ab_bench.sh ${1:-r03w}_ab b16
