#!/bin/bash
# C2 (lap2d 1000^2) level log and profile
set -o pipefail
OUT=gpurun_out/${1:-r05c2}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload lap2d --nx 1000 --no-cpu --no-abi --no-next --level-log --steps 3 > $OUT/lap2d.json 2> $OUT/lap2d.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --workload lap2d --nx 1000 --no-cpu --no-abi --no-next --roofline-only --warmup 0 > $OUT/prof.json 2> $OUT/prof.err && \
python3 tools/rocprof_summary.py $OUT/prof > $OUT/rocprof_stats.txt && rm -rf $OUT/prof && head -16 $OUT/rocprof_stats.txt && python3 -c "import json; d=json.load(open('$OUT/lap2d.json')); print(d['ms_per_step'], d['phases_ms_per_step_rank0'])"
