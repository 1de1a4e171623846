#!/bin/bash
# Round-6 diagnostics: k_diag_strips phase probe (w = 256), per-tile
# k_schur_big stamps of one 100^3 factorization, product bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 120 ./tools/micro/diag_strips_micro 256 1 5 > $O/ds_micro.txt 2>&1 && \
timeout -k 10 120 ./tools/micro/diag_strips_micro 256 8 5 >> $O/ds_micro.txt 2>&1 && cat $O/ds_micro.txt && \
SLU_LIB=ablib/stamp/libslu_mi355x_full.so SLU_STAMP_OUT=$O/stamps.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --no-next --no-abi > $O/bench_stamp.json 2> $O/bench_stamp.err && \
timeout -k 10 200 python tools/stamp_analyze.py $O/stamps.bin > $O/stamps.txt 2>&1 && rm -f $O/stamps.bin && cat $O/stamps.txt && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-next --no-abi > $O/bench.json 2> $O/bench.err && \
python -c "import json; d=json.load(open('$O/bench.json')); print('ms_per_step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'launch_ms', d['roofline']['avg_launch_ms'], 'serial', d['roofline']['serial_factor_ms'])"
