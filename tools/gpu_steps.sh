#!/bin/bash
# Run GPU steps in order on the gpurun box; stop after any step whose exit status signals a fault,
# abort, segfault or time limit (anything but 0 = ok / 1 = ordinary test failure).
# usage: tools/gpu_steps.sh "<name>:<timeout_s>:<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (timeout ${tmo}s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: $name exited $rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
