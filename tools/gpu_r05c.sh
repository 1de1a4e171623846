#!/bin/bash
# Round 5 GPU session c.  Each step has its own time limit; an ordinary
# failure (exit 1) is recorded and the session goes on, a time limit, abort or
# signal (exit >= 124) ends it.
OUT=gpurun_out/${1:-r05c}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
step() { # name limit cmd...
    local name=$1 lim=$2; shift 2
    echo "== $name"
    timeout -k 10 $lim "$@" > $OUT/$name.out 2> $OUT/$name.err
    local rc=$?
    echo "   rc=$rc"; tail -4 $OUT/$name.out
    if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi
    return 0
}
step pytest_regrid 500 python -u -m pytest tests/test_dropin.py -m gpu -v --timeout 300 --timeout-method thread \
    -k "evicts or without_plan_cache or device_resident"
step pytest_symb 300 python -u -m pytest tests/test_symbolic.py -m gpu -q --timeout 120 --timeout-method thread
step pytest_grid 700 python -u -m pytest tests/test_grid.py -m gpu -q -x --timeout 300 --timeout-method thread \
    -k "grid_matches or fingerprints"
step rehearse_n4 400 python -u bench.py --gpus 4 --host-transport --nx 40 --steps 2 --warmup 1
step bench_levels 400 python -u bench.py --no-cpu --no-abi --no-next --level-log --steps 1 --warmup 1
step bench_graph 500 python -u bench.py --ordering graph --no-cpu --no-abi --no-next --steps 2 --warmup 1
echo "== done"
