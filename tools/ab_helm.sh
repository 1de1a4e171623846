set -o pipefail
for r in 1 2; do for v in base rmw; do lib=""; [ $v != base ] && lib=ablib/$v/libslu_mi355x.so
SLU_LIB=$lib timeout -k 10 400 python -u bench.py --workload helm3d --steps 3 --warmup 1 --no-next --no-abi > gpurun_out/h_$v.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/h_$v.json')); r=d['roofline']; print('helm3d $v', d['ms_per_step'], r['frac'], r['serial_factor_ms'])"; done; done
