#!/bin/bash
# Retry gpurun while no box/slot is free (nothing ran, nothing charged); stop on any other outcome.
out=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  ec=$?
  if grep -q "status=transient" "$out" || [ $ec = 3 ]; then
    echo "attempt $i: no box ($ec), waiting" >> "$out.attempts"
    sleep 150
    continue
  fi
  break
done
exit $ec
