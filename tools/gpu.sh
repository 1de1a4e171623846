#!/bin/bash
# gpurun wrapper: retries ONLY when gpurun reports an infrastructure-side
# transient failure (nothing ran, nothing charged).  Usage: tools/gpu.sh LIMIT 'cmd'
limit=$1; shift
for attempt in 1 2 3 4; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$limit" -- "$@" 2>&1)
  echo "$out" | grep -v "^\s*$" | tail -4
  if echo "$out" | grep -q "status=transient\|backing off\|no box or slot"; then
    sleep 30; continue
  fi
  break
done
