#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh r05smax "s32:SLU_DIAG_STRIPS_MAX=32" "s64:SLU_DIAG_STRIPS_MAX=64" "s128:SLU_DIAG_STRIPS_MAX=128"
