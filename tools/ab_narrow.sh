set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/narrow; mkdir -p $O
SLU_LIB=ablib/narrow/libslu_mi355x.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_refdump.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_bench.sh narrow_ab narrow || exit 1
SLU_LIB=ablib/stampn/libslu_mi355x.so SLU_STAMP_OUT=$O/stamps.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --no-next --no-abi > $O/bench_stamp.json 2> $O/bench_stamp.err && \
timeout -k 10 200 python tools/stamp_analyze.py $O/stamps.bin > $O/stamps.txt 2>&1 && rm -f $O/stamps.bin && cat $O/stamps.txt
