#!/bin/bash
# Round 4: streamed upload on/off alternating on the cached drop-in call, with
# the D2H pipeline's own timing.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04q; rm -rf $O; mkdir -p $O
SUPERLU_MI355X_TIMING=1 SLU_PROFILE_PLAN=1 timeout -k 10 600 python -u tools/d2h_variants.py 100 stream > $O/var.txt 2> $O/var.err || { tail -20 $O/var.err; exit 1; }
cat $O/var.txt; grep -E "^rep|PDGSTRF|slu d2h|slu stream" $O/var.err | tail -30
