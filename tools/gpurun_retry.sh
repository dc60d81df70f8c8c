#!/bin/bash
# Submit one gpurun call; if no GPU slot is free (gpurun exit 3: nothing ran, nothing charged) wait and submit the
# same call again, at most $TRIES times.  Any other exit code (including a failed GPU step) ends it at once.
#   usage: tools/gpurun_retry.sh <log> <timeout-seconds> '<command>'
log=$1; secs=$2; cmd=$3; tries=${TRIES:-12}
for i in $(seq 1 $tries); do
  /usr/local/graft/bin/gpurun --timeout "$secs" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "slot(s) on this pod are busy" "$log"; then break; fi
  sleep 200
done
echo "gpurun rc=$rc after $i tries" >> "$log"
