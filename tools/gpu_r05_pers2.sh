#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh ${1:-r05p2} "big:SLU_SB_PERSIST=0" "pers:SLU_SB_PERSIST=1" "persnopf:SLU_SB_PERSIST=2"
