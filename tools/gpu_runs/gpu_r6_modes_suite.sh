#!/bin/bash
# Round 6: the whole GPU suite with each record source forced for every binned launch
# (SRT_TRACE_RECORDS=recompute, then =stored), beside the default policy's run in final2/.
source "$(dirname "$0")/gpu_lib.sh"
SRT_TRACE_RECORDS=recompute run suite_recompute 900 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread
tail -1 gpurun_out/suite_recompute.log
SRT_TRACE_RECORDS=stored run suite_stored 900 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread
tail -1 gpurun_out/suite_stored.log
