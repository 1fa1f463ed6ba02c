#!/bin/bash
# Round-6 session: the BASELINE configs' code paths over a 1-rank RCCL group
# (KFB_FORCE_PG=1): VGG-16 with fp16 gradient all-reduce, ResNet-152 bs32
# PairAveraging, ResNet-50 SMA / ada_sgd.  Each GPU step under its own time
# limit; fault / abort / timeout stops the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r13q"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {
  local name="$1" to="$2"; shift 2
  echo "== $name (limit ${to}s)"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "$OUT/$name.log" | cut -c1-700
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
B="python bench.py --steps 10 --warmup 5"
step vgg16_fp16wire 300 env KFB_FORCE_PG=1 $B --model vgg16 --batch_size 128 --wire_dtype fp16
step resnet152_pair 300 env KFB_FORCE_PG=1 $B --model resnet152 --batch_size 32 --kungfu_option async_sgd
step resnet50_sma 300 env KFB_FORCE_PG=1 $B --kungfu_option sma
step resnet50_ada 300 env KFB_FORCE_PG=1 $B --kungfu_option ada_sgd
echo done
