#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool gave no box
# (exit 3 / status=transient: nothing ran, nothing charged); any call that
# ran -- passed or failed -- ends the loop.  At most 10 submissions, 90 s apart.
# usage: tools/gpurun_queue.sh <log> <timeout> <command>
log=$1; to=$2; shift 2
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if grep -q "run [1-9][0-9.]*s of limit" "$log"; then exit $rc; fi
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$log"; then exit $rc; fi
  sleep 90
done
exit $rc
