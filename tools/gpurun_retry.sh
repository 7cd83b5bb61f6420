#!/bin/bash
# Runs one gpurun call; while the pool reports no box / a transient infrastructure failure
# (nothing ran, nothing charged) waits and asks again, at most 8 times.  A call that ran is
# never repeated.   tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|backing off\|slot(s) on this pod are busy" $LOG && ! grep -q "status=ok\|status=fail" $LOG; then
    sleep 90; continue
  fi
  exit $rc
done
exit 3
