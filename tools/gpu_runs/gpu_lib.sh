#!/bin/bash
# Shared helper for GPU-box scripts: `run NAME TIMEOUT CMD...` runs one GPU step under its own
# time limit with output in gpurun_out/NAME.log; a crash-type exit (fault, abort, segfault,
# timeout: anything but 0 or 1) ends the calling script, test failures (1) do not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "${BASH_SOURCE[0]}")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
}
