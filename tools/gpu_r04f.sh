#!/bin/bash
# Round 4: the other BASELINE configurations on the structure pdgssvx builds
# (reference symbfact + pddistribute; the plans amalgamate it): C2 lap2d
# 1000^2, C5 st27 120^3 fp32, C4 helm3d 80^3 complex on one GPU, then C4 as a
# 2x2 rehearsal on one GPU through the host transport (not a measurement).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04f; mkdir -p $O
for w in lap2d st27 helm3d; do
  timeout -k 10 600 python -u bench.py --workload $w --steps 5 --warmup 2 --no-next --no-abi > $O/$w.json 2> $O/$w.err || { echo "FAILED $w"; tail -20 $O/$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$w.json')); r=d['roofline']; c=d['config']; print('$w', d['ms_per_step'], d['value'], r['frac'], r['avg_launch_ms'], c['nsupers'], c['nsupers_factored'])"
done
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29514 bench.py --gpus 4 --steps 2 --warmup 1 --host-transport --workload helm3d \
    > $O/helm3d_2x2.json 2> $O/helm3d_2x2.err || { echo "FAILED helm3d 2x2"; tail -20 $O/helm3d_2x2.err; exit 1; }
python -c "import json; L=open('$O/helm3d_2x2.json').read().splitlines(); d=json.loads(L[-1]); c=d['config']; print('helm3d 2x2', d['ms_per_step'], d['value'], c['grid'], c['nsupers'], c['nsupers_factored'])"
