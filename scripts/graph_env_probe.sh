#!/bin/bash
# HIP-graph replay vs eager for the ResNet-50 step under HIP graph-execution
# knobs (does graph replay keep the weight-gradient side stream concurrent?).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/graphenv; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # tag bs env...
  local tag=$1 bs=$2; shift 2
  echo "== $tag bs$bs $*"
  env "$@" timeout -k 10 300 python scripts/graph_probe.py $bs > $OUT/$tag.$bs.log 2>&1
  local rc=$?; tail -n 3 $OUT/$tag.$bs.log
  case $rc in 0) ;; *) echo "rc=$rc, stopping"; exit $rc;; esac
}
run default 64 X=1
run queues4 64 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
run nopkt 64 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run nopkt_q4 64 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
run default 256 X=1
run queues4 256 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
run nopkt 256 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
