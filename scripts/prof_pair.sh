#!/bin/bash
# Kernel-trace two env variants of the bench with every kernel serialized on
# one stream (KFB_WGRAD_STREAM=0), so per-kernel times are comparable:
#   usage: scripts/prof_pair.sh <tag> "<env A>" "<env B>" [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; A="$2"; B="$3"; shift 3
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in A B; do
  if [ "$v" = A ]; then E="$A"; else E="$B"; fi
  for kv in $E; do export "$kv"; done
  export KFB_WGRAD_STREAM=0
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof$v" -o run -- \
      python3 "$ROOT/bench.py" --steps 6 --warmup 6 "$@" > "$OUT/prof$v.log" 2>&1 || exit $?
  for kv in $E; do unset "${kv%%=*}"; done
  f=$(find "$OUT/prof$v" -name "*kernel_trace.csv" | head -n 1)
  python3 "$ROOT/scripts/kernel_stats.py" "$f" --last-steps 4 --top 40 > "$OUT/kernels_$v.txt"
  rm -rf "$OUT/prof$v"
  echo "$v ($E): $(head -n 1 "$OUT/kernels_$v.txt")"
done
