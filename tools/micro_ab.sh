set -o pipefail
O=gpurun_out/micro1; mkdir -p $O
for v in atom rmw; do echo "== $v"; timeout -k 5 60 tools/micro/schur_micro_$v 8192 8192 256 4 || exit 1; done > $O/out.txt 2>&1
echo "== rmw ATOMIC=1" >> $O/out.txt; ATOMIC=1 timeout -k 5 60 tools/micro/schur_micro_rmw 8192 8192 256 4 >> $O/out.txt 2>&1
cat $O/out.txt
