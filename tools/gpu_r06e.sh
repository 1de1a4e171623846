#!/bin/bash
# Round 6: the whole GPU suite on the chunked-exchange tree, the 2- and
# 4-rank host-transport rehearsals (parity preflight), the N=1 bench line
# without the CPU leg (drop-in device-resident first-call figures).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06e}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --steps 2 --warmup 1 --host-transport --nx 60 \
      > $O/rehearse_n$n.json 2> $O/rehearse_n$n.err || { echo "FAILED n=$n"; tail -20 $O/rehearse_n$n.err; exit 1; }
  python -c "import json; L=open('$O/rehearse_n$n.json').read().splitlines(); d=json.loads(L[-1]); print('n=$n', d['ms_per_step'], d['value'], d['config']['grid'], d['config']['transport'], d.get('parity'))"
done
timeout -k 10 600 python -u bench.py --no-cpu --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac']); print(json.dumps(d.get('abi_pdgstrf',{}).get('device_resident',{}))[:1500])"
