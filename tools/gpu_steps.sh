#!/bin/bash
# Run GPU steps in order, each under its own time limit, output to
# gpurun_out/<name>.log:
#     tools/gpu_steps.sh NAME SECONDS 'COMMAND' [NAME SECONDS 'COMMAND' ...]
# A step that fails with an ordinary error (e.g. a test assertion, rc 1-2)
# does not stop the later steps; a time limit (124/137), an abort (134), a
# segfault (139) or any other signal death stops the whole run right there:
# nothing else touches the GPU after a possible fault.
mkdir -p gpurun_out
rc_all=0
while [ $# -ge 3 ]; do
    name=$1; secs=$2; cmd=$3; shift 3
    echo "[steps] $name (limit ${secs}s): $cmd"
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "[steps] $name rc=$rc in $(( $(date +%s) - start ))s"
    tail -3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then rc_all=$rc; fi
    if [ $rc -ge 124 ]; then
        echo "[steps] stopping: $name ended with $rc (time limit / abort / signal)"
        exit $rc
    fi
done
exit $rc_all
