#!/bin/bash
# Run one gpurun call, waiting while the pool has no free box or slot.
#   tools/gpurun_when_free.sh OUTFILE -- gpurun arguments...
# Only gpurun's exit code 3 ("no box or slot free right now, nothing
# charged": no part of the command ran) is waited out, up to GPURUN_TRIES (40) times, 2
# minutes apart.  Any other outcome -- including a failed GPU step -- ends it.
out=$1; shift; [[ $1 == -- ]] && shift
for i in $(seq ${GPURUN_TRIES:-40}); do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  [[ $rc -ne 3 ]] && break
  echo "[gpurun_when_free] no free box (try $i), waiting" >> "$out.wait"
  sleep 120
done
echo "exit $rc" >> "$out"
exit $rc
