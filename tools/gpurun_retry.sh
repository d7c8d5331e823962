#!/bin/bash
# gpurun with retries on infrastructure failures that happen before the command runs
# usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for a in 1 2 3 4; do
  timeout $((TO + 1200)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if grep -q "stopped responding while being prepared\|backing off\|status=transient" $LOG || [ $rc -eq 3 ]; then
    echo "[retry $a after infra failure rc=$rc]" >> $LOG.retries; sleep 45; continue
  fi
  break
done
echo "done rc=$rc" >> $LOG
