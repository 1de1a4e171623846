#!/bin/bash
# Regenerates tests/golden/abi_layout.json from the reference headers.
# Needs /root/reference (this container only).  Test infrastructure.
set -euo pipefail
here=$(cd "$(dirname "$0")" && pwd)
repo=$(cd "$here/../.." && pwd)
tmp=$(mktemp -d)
MPICH_CC=gcc /opt/conda/bin/mpicc -DREF -I/root/reference/SRC -I"$here" "$here/abi_probe.c" -o "$tmp/probe"
"$tmp/probe" | python3 -m json.tool > "$repo/tests/golden/abi_layout.json"
rm -rf "$tmp"
echo "wrote $repo/tests/golden/abi_layout.json"
