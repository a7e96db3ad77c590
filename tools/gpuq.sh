#!/bin/bash
# (round 5) queue a gpurun call: retry only while no GPU slot/box is free (exit 3: nothing ran, nothing charged)
log=$1; shift
for i in $(seq 1 20); do
  timeout 1500 /usr/local/graft/bin/gpurun --timeout "$GT" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$log"; then break; fi
  sleep 120
done
echo "GPUQ_RC=$rc tries=$i" >> "$log"
