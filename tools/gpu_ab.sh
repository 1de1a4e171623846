#!/bin/bash
# A/B session: parity subset (optionally with env for the candidate), then
# the 100^3 bench with the serialized level log for each env setting.
# usage: TAG=name ENVS="A=1 A=0" [SKIP_TESTS=1] bash tools/gpu_ab.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_refdump.py tests/test_grid.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for e in ${ENVS:-X=0}; do
  n=$(echo "$e" | tr '/=' '_-')
  env $e timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-next --no-abi --level-log > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$n.json')); print('$e', 'ms_per_step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'serial', d['roofline']['serial_factor_ms'])"
done
