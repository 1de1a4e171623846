#!/bin/bash
# End-of-round: the round script (whole GPU suite, bench, rocprof, PMC) on the
# headline workload, then the other BASELINE workloads' bench lines and the
# drop-in device-resident first call.  usage: bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-r06final}
bash tools/gpu_round.sh $TAG || exit 1
O=gpurun_out/$TAG
for w in st27 helm3d lap2d; do
  echo "== bench $w"
  timeout -k 10 600 python -u bench.py --workload $w --no-next --no-abi > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
done
echo "== done all"
