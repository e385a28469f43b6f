#!/bin/bash
# Run one gpurun call, retrying only while the pool has no free box (exit 3: nothing ran, nothing
# charged).  Usage: tools/gpu_retry.sh LOG gpurun-args...
out=$1; shift
for i in $(seq 1 30); do
    /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
    rc=$?
    [ $rc -ne 3 ] && exit $rc
    sleep 100
done
exit 3
