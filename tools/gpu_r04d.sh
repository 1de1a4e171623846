#!/bin/bash
# Round 4: k_diag_strips micro, its parity tests, then a short 100^3 bench
# (no CPU baseline) for the factor time with the strips on the panel stream.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O; rm -f $O/micro.txt
for a in "256 1" "256 4" "128 1" "64 1"; do
  timeout -k 10 60 ./tools/micro/diag_strips_micro $a 5 >> $O/micro.txt 2>&1 || { echo "FAIL $a rc=$?" >> $O/micro.txt; cat $O/micro.txt; exit 1; }
done
cat $O/micro.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_refdump.py -m gpu -x -v -k "strips or dropin_pdgstrf or reference_structure" \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cpu > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
