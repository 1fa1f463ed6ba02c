#!/bin/bash
# PMC counter passes over representative conv layers (HIP kernels only).
# usage: scripts/pmc_conv.sh <tag> [shape indices]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-pmc}"; SHAPES="${2:-1,4,12,13}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  echo "== pass $i: $set"
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/scripts/bench_conv.py" --iters 2 --hip_only --shapes "$SHAPES" \
      > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  case $rc in 0) ;; *) tail -n 5 "$OUT/p$i.log"; [ $rc -ge 124 ] && exit $rc;; esac
  f=$(find "$OUT/p$i" -name "*counter_collection.csv" | head -n 1)
  [ -n "$f" ] && python3 "$ROOT/scripts/pmc_summary.py" "$f" --filter kfb > "$OUT/summary_p$i.txt"
done
echo done
