#!/bin/bash
# zoo refresh (launch tape on, raw replay): usage gpu_zoo_r9.sh <tag> <part 1|2>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export KFB_TAPE_RAW=1 KFB_TAPE_PROFILE=1
if [ "${2:-1}" = 1 ]; then
  exec_models="resnet50:64 resnet152:32 inception4:64 resnet101:128 resnet152:128 resnet50_v1.5:256 resnet50_v2:256 official_resnet50:128 official_resnet152:64 inception3:128"
else
  exec_models="mobilenet:128 nasnet:64 googlenet:128 vgg11:128 vgg16:128 vgg19:128 alexnet:512 overfeat:256 nasnetlarge:16 trivial:256"
fi
bash scripts/zoo_bench.sh "$1" $exec_models
