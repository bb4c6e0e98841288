#!/bin/bash
# Calls gpurun with the given command, and calls it again only while gpurun answers
# "status=transient" (no box, a box lost while being prepared, or a backoff: nothing of the
# command ran and nothing was charged), waiting the time gpurun asks for. Any other outcome
# (the command ran, whatever its exit code) ends the loop.
#   bash nzcb-circom_amd/tools/gpurun_when_free.sh <log> <timeout_s> <command...>
log=$1; shift
limit=$1; shift
for attempt in $(seq 1 12); do
  timeout $((limit + 900)) /usr/local/graft/bin/gpurun --timeout "$limit" -- "$@" > "$log" 2>&1
  rc=$?
  if ! grep -q 'status=transient' "$log"; then
    exit $rc
  fi
  wait_s=$(grep -o 'retry in [0-9]*s' "$log" | grep -o '[0-9]*' | tail -1)
  [ -z "$wait_s" ] && wait_s=120
  echo "attempt $attempt transient; waiting $((wait_s + 15)) s" >> "$log.attempts"
  sleep $((wait_s + 15))
done
exit 75
