#!/bin/bash
# gpurun with retries when the call never ran: an infrastructure failure while the box
# was prepared, a back-off, or no free GPU slot (exit 3).  A command that ran is never
# repeated.  usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for a in $(seq 1 ${TRIES:-8}); do
  timeout $((TO + 1200)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "stopped responding while being prepared\|backing off\|status=transient" $LOG; then
    echo "[retry $a: the call did not run, rc=$rc]" >> $LOG.retries; sleep ${NAP:-120}; continue
  fi
  break
done
echo "done rc=$rc" >> $LOG
