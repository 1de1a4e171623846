#!/bin/bash
# Schur micro at small K: atomic scatter vs plain read-modify-write
set -o pipefail
for kw in 32 64 128 256; do
  echo "kw=$kw atomic:"; timeout -k 5 60 tools/micro/schur_micro_atom 8192 8192 $kw 3 | grep k_schur | tail -1 || exit 1
  echo "kw=$kw rmw:";    timeout -k 5 60 tools/micro/schur_micro_rmw 8192 8192 $kw 3 | grep k_schur | tail -1 || exit 1
done
