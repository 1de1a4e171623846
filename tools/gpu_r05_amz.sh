#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh ${1:-r05amz} "z10:SLU_AMALG_ZERO=0.10" "z05:SLU_AMALG_ZERO=0.05" "z15:SLU_AMALG_ZERO=0.15" "z20:SLU_AMALG_ZERO=0.20"
