#!/bin/bash
# Round 3: amalgamation follow-ups (merged D2H pieces, sorted coarse rows,
# reference-partition flops) -- the affected GPU tests, the headline bench
# without the CPU leg, and the grid rehearsal on the coarse reference partition.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_refdump.py tests/test_dropin.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && tail -2 $O/pytest.log && \
timeout -k 10 600 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err && cat $O/bench.json && \
for n in 2 4; do
  timeout -k 10 400 python -u bench.py --gpus $n --steps 2 --warmup 1 --host-transport --nx 60 \
      > $O/rehearse_n$n.json 2> $O/rehearse_n$n.err || { echo "FAILED n=$n"; tail -20 $O/rehearse_n$n.err; exit 1; }
  cat $O/rehearse_n$n.json
done
