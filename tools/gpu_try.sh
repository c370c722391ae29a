#!/bin/bash
# Retry a gpurun call only while the pool reports that nothing ran (transient: no slot / no box /
# box preparation failed; run 0 s, nothing charged).  Any call that ran is final.
# usage: tools/gpu_try.sh LOG TIMEOUT 'command'
log=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6 7 8; do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $log 2>&1
  if grep -q "status=transient" $log && grep -q "run 0.0s\|run Nones" $log; then
    echo "try $i: transient, nothing ran; waiting" >> $log.tries
    sleep 150
    continue
  fi
  break
done
tail -80 $log
