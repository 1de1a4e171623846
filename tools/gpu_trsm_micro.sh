set -e
mkdir -p gpurun_out/r06i
rm -f gpurun_out/r06i/trsm_probe.txt
for n in 1 4 64 256; do
  timeout -k 10 60 ./tools/micro/trsm_micro $n 20 >> gpurun_out/r06i/trsm_probe.txt
done
cat gpurun_out/r06i/trsm_probe.txt
