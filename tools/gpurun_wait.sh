#!/bin/bash
# Run a gpurun command, waiting while the pod has no free GPU slot (gpurun exit
# code 3 / "busy": nothing ran, nothing charged).  Any other outcome is returned.
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun "$@" 2>&1 | tee /tmp/gpurun_wait.out
  rc=${PIPESTATUS[0]}
  if [ $rc -ne 3 ] && ! grep -q "are busy\|no box\|retry in a few minutes" /tmp/gpurun_wait.out; then exit $rc; fi
  echo "[gpurun_wait] no slot free (rc=$rc), retry $i in 60 s" >&2
  sleep 60
done
exit 3
