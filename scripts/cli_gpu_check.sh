#!/bin/bash
# End-to-end CLI runs on one GPU (the tf_cnn_benchmarks.py surface a user
# switching from the reference would exercise): train with checkpoints,
# summaries and a Chrome trace, resume, eval from the checkpoint,
# forward-only, train-and-eval, real-data-format input (TFRecord fixture).
#   usage: scripts/cli_gpu_check.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="${1:-cli}"
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
TD="$OUT/train_dir"; rm -rf "$TD"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # run <name> <args...>
  local name="$1"; shift
  timeout -k 10 300 python tf_cnn_benchmarks.py "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -E 'total images/sec|Accuracy @ 1|examples/sec' "$OUT/$name.log" | tail -n 1)"
  case $rc in 0) ;; 124|134|137|139) echo "FATAL"; exit $rc;; *) tail -n 5 "$OUT/$name.log";; esac
}
COMMON="--model=resnet50 --batch_size=64 --use_bf16 --optimizer=momentum --num_warmup_batches=2 --display_every=5"
run train $COMMON --num_batches=10 --train_dir="$TD" --save_model_steps=5 --summary_verbosity=1 \
    --save_summaries_steps=5 --trace_file="$OUT/trace.json"
run resume $COMMON --num_batches=15 --train_dir="$TD"
run eval $COMMON --eval --train_dir="$TD" --num_eval_batches=3
run forward_only $COMMON --forward_only --num_batches=5
run train_and_eval $COMMON --num_batches=6 --train_dir="$OUT/td2" \
    --eval_during_training_every_n_steps=3 --num_eval_batches=2
python -c "from kf_benchmarks_amd.data import test_data; test_data.write_black_and_white_tfrecord_data('$OUT/fake_data', 11, num_train_images=256, num_validation_images=64)"
run real_data --model=resnet50 --batch_size=32 --use_bf16 --num_warmup_batches=1 --num_batches=5 \
    --data_dir="$OUT/fake_data" --data_name=imagenet --display_every=1
run inception3 --model=inception3 --batch_size=32 --use_bf16 --num_warmup_batches=1 --num_batches=4
run vgg16_fp16 --model=vgg16 --batch_size=32 --use_fp16 --fp16_enable_auto_loss_scale --num_warmup_batches=1 --num_batches=4
ls -la "$TD" > "$OUT/train_dir_listing.txt"
python -c "import json; d=json.load(open('$OUT/trace.json')); print('trace events', len(d.get('traceEvents', d)))" > "$OUT/trace_check.txt" 2>&1
# checkpoints / fixtures / traces are large: keep only logs and listings
rm -rf "$TD" "$OUT/td2" "$OUT/fake_data" "$OUT/trace.json"
echo done
