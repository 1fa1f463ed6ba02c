#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter set) over any python
# command; per-kernel means summarized by scripts/pmc_summary.py.
# usage: scripts/pmc_cmd.sh <tag> <kernel-name filter> <script.py> [args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; FLT="$2"; shift 2
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  echo "== pass $i: $set"
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/$1" "${@:2}" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  case $rc in 0) ;; *) tail -n 5 "$OUT/p$i.log"; exit $rc;; esac
  f=$(find "$OUT/p$i" -name "*counter_collection.csv" | head -n 1)
  [ -n "$f" ] && python3 "$ROOT/scripts/pmc_summary.py" "$f" --filter "$FLT" > "$OUT/summary_p$i.txt"
  rm -f "$OUT"/p$i/*/*kernel_trace.csv 2>/dev/null
done
echo done
