#!/bin/bash
# Store-stream calibration sweep (tools/probe/store_probe.hip); one process per case.
# args: worlds steps rows line3 cols valu rowaux wait
set -u
P=${GRAFT_REPO_ROOT:-.}/tools/probe/store_probe
for W in ${WORLDS:-32768 65536 262144}; do
  for cfg in "1 0 1 0 2 0" "0 0 0 256 2 0" "0 0 0 512 2 0" "1 0 1 256 2 0" "1 0 1 256 2 3" "1 0 1 512 2 0" "1 0 1 512 2 3" "1 0 0 256 2 0" "1 0 0 256 2 3"; do
    timeout -k 5 60 $P $W 1000 $cfg || exit $?
  done
done
