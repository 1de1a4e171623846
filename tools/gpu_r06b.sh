#!/bin/bash
# Round-6: k_trsm_wv (SLU_TRSM_WV=1) parity on the GPU parity / refdump /
# grid suites, A/B of the 100^3 factorization (serialized level log for the
# panel kernels), k_diag_strips phase probe, Schur stamps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
SLU_TRSM_WV=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_refdump.py tests/test_grid.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_wv.log 2>&1 || { tail -40 $O/pytest_wv.log; exit 1; }
tail -2 $O/pytest_wv.log
for v in 1 0; do
  SLU_TRSM_WV=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-next --no-abi --level-log > $O/bench_wv$v.json 2> $O/bench_wv$v.err || { tail -20 $O/bench_wv$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_wv$v.json')); print('wv=$v ms_per_step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'serial', d['roofline']['serial_factor_ms'])"
done
timeout -k 10 120 ./tools/micro/diag_strips_micro 256 1 5 > $O/ds_micro.txt 2>&1 && cat $O/ds_micro.txt
SLU_LIB=ablib/stamp/libslu_mi355x_full.so SLU_STAMP_OUT=$O/stamps.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --no-next --no-abi > $O/bench_stamp.json 2> $O/bench_stamp.err && \
timeout -k 10 200 python tools/stamp_analyze.py $O/stamps.bin > $O/stamps.txt 2>&1 && rm -f $O/stamps.bin && cat $O/stamps.txt
