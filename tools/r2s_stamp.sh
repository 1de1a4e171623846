#!/bin/bash
# Diagnostics session: parity tests, per-tile k_schur_big stamps of one 100^3
# factorization (diagnostics build ablib/stamp), and the product bench line.
# usage: bash tools/r2s_stamp.sh TAG [--no-tests]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2s}
O=gpurun_out/$TAG; mkdir -p $O
if [ "$2" != "--no-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
SLU_LIB=ablib/stamp/libslu_mi355x.so SLU_STAMP_OUT=$O/stamps.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --no-next --no-abi > $O/bench_stamp.json 2> $O/bench_stamp.err && \
timeout -k 10 200 python tools/stamp_analyze.py $O/stamps.bin > $O/stamps.txt 2>&1 && \
python -c "import numpy as np; a=np.fromfile('$O/stamps.bin',dtype=np.uint64).reshape(-1,4); a[::8].tofile('$O/stamps_s8.bin')" && rm -f $O/stamps.bin && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-next --no-abi > $O/bench.json 2> $O/bench.err && \
cat $O/stamps.txt && python -c "import json; d=json.load(open('$O/bench.json')); print('ms_per_step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'launch_ms', d['roofline']['avg_launch_ms'], 'serial', d['roofline']['serial_factor_ms'])"
# A/B: the same library with one workgroup per tile
SLU_SB_PERSIST=0 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-next --no-abi > $O/bench_np.json 2> $O/bench_np.err && \
python -c "import json; d=json.load(open('$O/bench_np.json')); print('non-persistent ms_per_step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'launch_ms', d['roofline']['avg_launch_ms'], 'serial', d['roofline']['serial_factor_ms'])"
