#!/bin/bash
# GPU suite (the driver's command) into gpurun_out/<tag>/gputest.log
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06_suite}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${2:-} > gpurun_out/$TAG/gputest.log 2>&1 || { tail -40 gpurun_out/$TAG/gputest.log; exit 1; }
tail -1 gpurun_out/$TAG/gputest.log
