#!/bin/bash
# Multi-rank rehearsal of bench.py on one GPU (host-staged transport, RCCL
# refuses two ranks on one device) + the other BASELINE workloads at N=1
# (WORKLOADS="" skips them).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/rehearse; mkdir -p $O
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --steps 2 --warmup 1 --host-transport --nx 60 \
      > $O/n$n.json 2> $O/n$n.err || { echo "FAILED n=$n"; tail -20 $O/n$n.err; exit 1; }
  python -c "import json; L=open('$O/n$n.json').read().splitlines(); assert len(L) == 1, L; d=json.loads(L[0]); print('n=$n', d['ms_per_step'], d['value'], d['config']['grid'], d['config']['transport'])"
done
for w in ${WORKLOADS-lap2d st27 helm3d}; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 3 --warmup 1 --no-next --no-abi > $O/$w.json 2> $O/$w.err || { echo "FAILED $w"; tail -20 $O/$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$w.json')); r=d['roofline']; print('$w', d['ms_per_step'], d['value'], r['frac'], r['kernel'])"
done
