set -o pipefail
O=gpurun_out/r06s; mkdir -p $O
for d in 1 0; do
SUPERLU_MI355X_DEFER_A=$d SUPERLU_MI355X_TIMING=1 timeout -k 10 400 python -u bench.py --device-resident-child --nx 100 > $O/devres_$d.json 2> $O/devres_$d.err || { tail -30 $O/devres_$d.err; exit 1; }
echo "== DEFER_A=$d"; grep -v "^\[slu rank" $O/devres_$d.err | head -60; cat $O/devres_$d.json
done
