#!/bin/bash
# tape host profiles with device-op counts (host-bound-candidate configs)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export KFB_TAPE_PROFILE=1
bash scripts/zoo_bench.sh "${1:-r10z}" inception4:64 resnet152:32 resnet50:64 nasnet:64
for f in gpurun_out/${1:-r10z}/*.log; do echo "$f"; grep "tape host time" "$f"; done
