#!/bin/bash
# Round 3: multi-rank bench paths rehearsed on one GPU (host point-to-point
# transport): 2D 1x2 and 2x2, 3D 1x1x2 and 1x1x4, at 60^3.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03s}; mkdir -p $O
timeout -k 10 300 python -u bench.py --gpus 2 --host-transport --nx 60 --no-cpu > $O/g2.json 2> $O/g2.err && cut -c1-400 $O/g2.json && \
timeout -k 10 300 python -u bench.py --gpus 4 --host-transport --nx 60 --no-cpu > $O/g4.json 2> $O/g4.err && cut -c1-400 $O/g4.json && \
timeout -k 10 300 python -u bench.py --gpus 2 --grid3d 1x1x2 --host-transport --nx 60 --no-cpu > $O/z2.json 2> $O/z2.err && cut -c1-400 $O/z2.json && \
timeout -k 10 300 python -u bench.py --gpus 4 --grid3d 1x1x4 --host-transport --nx 60 --no-cpu > $O/z4.json 2> $O/z4.err && cut -c1-400 $O/z4.json && \
python3 -c "import json; d=json.load(open('$O/z4.json')); print(d['layers3d'])"
