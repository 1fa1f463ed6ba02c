"""Flag registry, Params validation, batch/epoch math and LR schedules
(tcb/benchmark_cnn_test.py:888-1003, 1179-1233 reproduced with the
reference's expected values)."""

import pytest

from kf_benchmarks_amd import benchmark, flags, optim, params as P
from kf_benchmarks_amd.models import model_config
from kf_benchmarks_amd import datasets


def test_reference_flag_surface_present():
    names = list(flags.param_specs)
    assert len(names) >= P.REFERENCE_FLAG_COUNT
    for n in ["model", "batch_size", "num_gpus", "variable_update", "kungfu_option",
              "all_reduce_spec", "gradient_repacking", "use_fp16", "train_dir",
              "eval_during_training_every_n_steps", "trt_mode", "benchmark_test_id",
              "compact_gradient_transfer", "hierarchical_copy", "staged_vars"]:
        assert n in flags.param_specs
    spec = flags.param_specs["variable_update"]
    assert "kungfu" in spec.kwargs["enum_values"] and spec.default_value == "parameter_server"
    assert flags.param_specs["model"].default_value == "trivial"
    assert flags.param_specs["weight_decay"].default_value == 0.00004


def test_parse_flags_forms():
    v = flags.parse_flags(["--model=resnet50", "--batch_size", "64", "--nodistortions",
                           "--use_fp16", "--eval_during_training_at_specified_steps=1,5",
                           "--momentum=0.8"])
    assert v == {"model": "resnet50", "batch_size": 64, "distortions": False, "use_fp16": True,
                 "eval_during_training_at_specified_steps": ["1", "5"], "momentum": 0.8}
    assert flags.parse_flags(["--distortions=false"]) == {"distortions": False}


@pytest.mark.parametrize("argv", [["positional"], ["--bogus_flag=1"],
                                  ["--variable_update=nonsense"], ["--batch_size=abc"],
                                  ["--gradient_repacking=-1"]])
def test_parse_flags_errors(argv):
    with pytest.raises(flags.FlagError):
        flags.parse_flags(argv)


def test_make_params_bounds():
    with pytest.raises(ValueError):
        P.make_params(num_batches=100, gradient_repacking=-1)
    with pytest.raises(ValueError):
        P.make_params(gpu_memory_frac_for_testing=2.0)
    with pytest.raises(ValueError):
        P.make_params(variable_update="bogus")
    p = P.make_params(batch_size=5)
    assert p.batch_size == 5 and p.model == "trivial"
    p2 = P.remove_param_fields(p, ["batch_size"])
    assert not hasattr(p2, "batch_size")


def test_flags_argv_roundtrip():
    p = P.make_params(model="resnet50", num_batches=7, distortions=False, use_bf16=True)
    argv = P.params_to_argv(p)
    p2 = P.make_params_from_flags(argv)
    assert p2 == p


@pytest.mark.parametrize("kw", [
    dict(device="cpu", data_format="NCHW"),
    dict(num_epochs_per_decay=1),
    dict(minimum_learning_rate=0.1),
    dict(variable_update="horovod", num_gpus=2),
    dict(variable_update="kungfu", num_gpus=2),
    dict(variable_update="kungfu", job_name="worker"),
    dict(hierarchical_copy=True, num_gpus=1),
    dict(save_model_secs=10, save_model_steps=10),
    dict(eval_during_training_every_n_steps=1, eval_during_training_every_n_epochs=1.0),
    dict(eval_during_training_every_n_steps=1, eval=True),
    dict(stop_at_top_1_accuracy=0.5),
    dict(trt_mode="FP32"),
    dict(use_fp16=True, fp16_vars=True, gradient_repacking=2),
    dict(staged_vars=True, variable_update="replicated"),
    dict(eval=True, forward_only=True),
    dict(use_fp16=True, use_bf16=True),
])
def test_invalid_flag_combinations(kw):
    with pytest.raises(ValueError):
        benchmark.validate_params_combinations(P.make_params(**kw))


def test_num_batches_and_epochs():
    p = P.make_params()
    b, e = benchmark.get_num_batches_and_epochs(p, 10, 100)
    assert b == benchmark._DEFAULT_NUM_BATCHES and e == pytest.approx(10.0)
    b, e = benchmark.get_num_batches_and_epochs(P.make_params(num_batches=21), 25, 50)
    assert b == 21 and e == pytest.approx(10.5)
    b, e = benchmark.get_num_batches_and_epochs(P.make_params(num_epochs=3), 2, 3)
    assert b == 4 and e == pytest.approx(8.0 / 3.0)
    with pytest.raises(ValueError):
        benchmark.get_num_batches_and_epochs(P.make_params(num_batches=100, num_epochs=100), 1, 1)


def _lr(params, steps):
    ds = datasets.create_dataset(None, "imagenet")
    model = model_config.get_model_config(params.model, ds, params)
    if params.batch_size:
        model.set_batch_size(params.batch_size)
    bs = model.get_batch_size() * params.num_gpus
    for step, want in steps.items():
        got = optim.get_learning_rate(params, step, ds.num_examples_per_epoch("train"), model, bs)
        assert got == pytest.approx(want, rel=1e-6, abs=1e-12), (step, got, want)


def test_lr_model_specific_resnet():
    p = P.make_params(model="resnet50", batch_size=256, variable_update="parameter_server",
                      num_gpus=1)
    _lr(p, {0: 0, 150136: 0.128, 150137: 0.0128, 300273: 0.0128, 300274: 0.00128,
            10000000: 0.0000128})


def test_lr_user_init():
    p = P.make_params(model="resnet50", batch_size=256, variable_update="replicated",
                      init_learning_rate=1.0)
    _lr(p, {0: 1.0, 10000000: 1.0})


def test_lr_user_init_and_warmup():
    p = P.make_params(model="resnet50", batch_size=256, variable_update="replicated",
                      init_learning_rate=1.0, num_learning_rate_warmup_epochs=5)
    _lr(p, {0: 0.0, 12511: 0.5, 25022: 1.0, 10000000: 1.0})


def test_lr_user_decay():
    p = P.make_params(model="resnet50", init_learning_rate=1.0, learning_rate_decay_factor=0.5,
                      num_epochs_per_decay=2, minimum_learning_rate=0.375, batch_size=32)
    _lr(p, {0: 1.0, 80071: 1.0, 80072: 0.5, 160143: 0.5, 160144: 0.375, 10000000: 0.375})


def test_lr_zero_decay_is_invalid():
    p = P.make_params(model="resnet50", num_learning_rate_warmup_epochs=0,
                      learning_rate_decay_factor=0.5, num_epochs_per_decay=0,
                      minimum_learning_rate=0.375, batch_size=32)
    with pytest.raises(ValueError):
        benchmark.validate_params_combinations(p)


def test_lr_piecewise_schedule():
    p = P.make_params(model="trivial", batch_size=32,
                      piecewise_learning_rate_schedule="1;3;.1;5;.01")
    _lr(p, {0: 1.0, 120108: 1.0, 120109: 0.1, 200181: 0.1, 200182: 0.01, 100000000: 0.01})


def test_piecewise_schedule_errors():
    with pytest.raises(ValueError):
        optim.get_piecewise_learning_rate("1;3", 0, 10)
    with pytest.raises(ValueError):
        optim.get_piecewise_learning_rate("1;x;2", 0, 10)
    with pytest.raises(ValueError):
        optim.get_piecewise_learning_rate("1;5;.1;3;.01", 0, 10)


@pytest.mark.parametrize("num_gpus,vu,lr", [(1, "parameter_server", 0.128), (2, "replicated", 0.064),
                                            (8, "replicated", 0.016),
                                            (8, "parameter_server", 0.128)])
def test_resnet_lr_scaling(num_gpus, vu, lr):
    """tcb/models/resnet_model_test.py: base LR scales with batch, /num_gpus in replicated."""
    from kf_benchmarks_amd.models import resnet_model
    p = P.make_params(model="resnet50", variable_update=vu, num_gpus=num_gpus)
    m = resnet_model.create_resnet50_model(p)
    assert m.get_scaled_base_learning_rate(256) == pytest.approx(lr)
