#!/bin/bash
# Round 4: the 100^3 level log (serialized kernel times per level, for
# tools/scale_model.py), then multi-rank rehearsals on one GPU through the
# host transport -- not measurements -- on the reference structure: the grid
# plans amalgamate it (nsupers_factored < nsupers).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-abi --no-next --level-log \
    > $O/level_bench.json 2> $O/level_log.txt || { tail -5 $O/level_log.txt; exit 1; }
cut -c1-300 $O/level_bench.json
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --steps 2 --warmup 1 --host-transport --nx 60 \
      > $O/rehearse_n$n.json 2> $O/rehearse_n$n.err || { echo "FAILED n=$n"; tail -20 $O/rehearse_n$n.err; exit 1; }
  python -c "import json; L=open('$O/rehearse_n$n.json').read().splitlines(); d=json.loads(L[-1]); c=d['config']; print('n=$n', d['ms_per_step'], d['value'], c['grid'], c['nsupers'], c['nsupers_factored'], c['transport'])"
done
