"""MobileNet-v2, official ResNets and NASNet: parameter counts against the
published architectures and a CPU forward/backward."""

import pytest
import torch

from kf_benchmarks_amd import datasets, params as P
from kf_benchmarks_amd.models import model_config
from kf_benchmarks_amd.models.model import make_network


def _net(name, ds="imagenet", size=None):
    d = datasets.create_dataset(None, ds)
    m = model_config.get_model_config(name, d, P.make_params(model=name))
    if size:
        m.image_size = size
    return d, m, make_network(m, d.num_classes, "cpu", torch.float32)


# published parameter counts (+ the CNNModel's final 1001/11-way affine)
@pytest.mark.parametrize("name,ds,expected", [
    ("mobilenet", "imagenet", 3.504e6 + 1001 * 1001 + 1001),
    ("official_resnet18", "imagenet", 11.69e6), ("official_resnet34", "imagenet", 21.80e6),
    ("official_resnet50", "imagenet", 25.56e6), ("official_resnet101_v2", "imagenet", 44.55e6),
    ("nasnet", "imagenet", 5.29e6), ("nasnet", "cifar10", 3.35e6)])
def test_param_counts(name, ds, expected):
    _, _, net = _net(name, ds)
    assert abs(net.num_params() - expected) / expected < 0.02, net.num_params()


@pytest.mark.parametrize("name,ds,size", [("mobilenet", "imagenet", 64),
                                          ("official_resnet18_v2", "imagenet", 64),
                                          ("nasnet", "cifar10", None)])
def test_forward_backward(name, ds, size):
    d, m, net = _net(name, ds, size)
    x = torch.randn(2, m.image_size, m.image_size, 3)
    y = torch.randint(0, d.num_classes - 1, (2,))
    res = net(x)
    loss = m.loss_function((x, y), res)
    loss.backward()
    assert torch.isfinite(loss)
    grads = [p.grad for _, p in net.trainable_variables()]
    assert all(g is not None and torch.isfinite(g).all() for g in grads)


def test_mobilenet_block_structure():
    _, _, net = _net("mobilenet")
    names = [n for n, _ in net.trainable_variables()]
    assert sum("depthwise_weights" in n for n in names) == 17
    # first block has no expansion conv; later ones do
    assert not any(n.startswith("MobilenetV2/expanded_conv/expand") for n in names)
    assert any(n.startswith("MobilenetV2/expanded_conv_1/expand") for n in names)


def test_ncf_engine_cpu():
    import kfb_test_util as tu
    from kf_benchmarks_amd import benchmark
    params = benchmark.make_params(model="ncf", batch_size=64, num_batches=3,
                                   num_warmup_batches=0, device="cpu", data_format="NHWC",
                                   optimizer="adam", weight_decay=0, display_every=1)
    with tu.capture_logs() as logs:
        stats = benchmark.BenchmarkCNN(params).run()
    assert stats["num_steps"] == 3
    losses = [o.loss for o in tu.get_training_outputs_from_logs(logs, False)]
    assert all(0 < l < 5 for l in losses)


def test_deepspeech2_small():
    from kf_benchmarks_amd import optim
    from kf_benchmarks_amd.models import deepspeech
    d, m, _ = _net("resnet20", "cifar10")  # dataset only
    d = datasets.create_dataset(None, "librispeech")
    m = model_config.get_model_config("deepspeech2", d, P.make_params(model="deepspeech2"))
    m.max_time_steps, m.max_label_length, m.rnn_hidden_size = 120, 20, 32
    m.set_batch_size(2)
    net = make_network(m, d.num_classes, "cpu", torch.float32)
    optim.FlatParams(net)
    inp = m.get_synthetic_inputs("x", d.num_classes, "cpu", 0)
    res = net.forward_inputs(inp)
    assert res.logits.shape == (2, 30, 29)
    loss = m.loss_function(inp, res)
    loss.backward()
    assert torch.isfinite(loss)
    r = m.postprocess({k: v.detach().numpy() for k, v in m.accuracy_function(inp, res.logits).items()})
    assert 0 <= r["cer"]
    dec = deepspeech.DeepSpeechDecoder()
    assert dec.decode([1, 1, 28, 1, 2, 2, 28]) == "aab"
    assert deepspeech.edit_distance("kitten", "sitting") == 3


def test_ssd300_loss_and_targets():
    import numpy as np
    from kf_benchmarks_amd.models import coco_metric, ssd_dataloader as sd
    assert sd.default_boxes()("ltrb").shape == (8732, 4)
    assert len(sd.CLASS_INV_MAP) == 81 and sd.CLASS_MAP[90] == 80
    gt = np.array([[0.1, 0.2, 0.5, 0.6], [0.3, 0.3, 0.9, 0.8]], np.float32)
    lab = np.array([[3], [7]], np.float32)
    c, b, n = sd.encode_labels(gt, lab)
    pos = c[:, 0] > 0
    assert n == pos.sum() >= 2 and set(np.unique(c)) == {0.0, 3.0, 7.0}
    dec = sd.decode_boxes(b, sd.default_boxes()("xywh"))
    sc = np.zeros((8732, 81), np.float32)
    sc[:, 0] = 1
    sc[pos] = 0
    sc[pos, c[pos, 0].astype(int)] = 1
    gtb = np.zeros((200, 4), np.float32)
    gtc = np.zeros((200, 1), np.float32)
    gtb[:2], gtc[:2] = gt, lab
    m = coco_metric.compute_map([dict(pred_boxes=dec, pred_scores=sc, gt_boxes=gtb,
                                      gt_classes=gtc)])
    assert m["AP"] > 0.99
    d = datasets.create_dataset(None, "coco")
    model = model_config.get_model_config("ssd300", d, P.make_params(model="ssd300",
                                                                     data_name="coco"))
    model.set_batch_size(2)
    net = make_network(model, d.num_classes, "cpu", torch.float32)
    inp = model.get_synthetic_inputs("x", 81, "cpu", 0)
    res = net.forward_inputs(inp)
    assert res.logits.shape == (2, 8732, 85)
    loss = model.loss_function(inp, res)
    loss.backward()
    assert torch.isfinite(loss)
    assert not model.l2_param_filter("resnet34_backbone/conv0/batchnorm0/gamma")
