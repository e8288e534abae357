#!/bin/bash
# (host side) one gpurun call, retried only while the pool has no box free
# (status=transient: nothing ran, nothing charged); usage: tools/gpu_try.sh CMD
# retries a gpurun call only while the pool has no box free (nothing ran)
for i in 1 2 3 4 5 6 7 8; do
  out=$(timeout 3000 /usr/local/graft/bin/gpurun --timeout ${GT:-1200} -- "$@" 2>&1)
  echo "$out" | tail -4
  if echo "$out" | grep -q "status=transient"; then sleep 150; continue; fi
  break
done
