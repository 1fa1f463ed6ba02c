"""Model registry (role of tcb/models/model_config.py:38-142).

Unlike the fork (which commented out everything but ResNet), every model of
the zoo is registered.  Models are imported lazily so a broken optional
family cannot break the others.
"""

from __future__ import annotations

import importlib


def _lazy(module, fn):
    def ctor(params):
        mod = importlib.import_module("kf_benchmarks_amd.models." + module)
        return getattr(mod, fn)(params=params)
    ctor.__name__ = fn
    return ctor


_IMAGENET = {
    "vgg11": _lazy("vgg_model", "Vgg11Model"),
    "vgg16": _lazy("vgg_model", "Vgg16Model"),
    "vgg19": _lazy("vgg_model", "Vgg19Model"),
    "lenet": _lazy("lenet_model", "Lenet5Model"),
    "googlenet": _lazy("googlenet_model", "GooglenetModel"),
    "overfeat": _lazy("overfeat_model", "OverfeatModel"),
    "alexnet": _lazy("alexnet_model", "AlexnetModel"),
    "trivial": _lazy("trivial_model", "TrivialModel"),
    "inception3": _lazy("inception_model", "Inceptionv3Model"),
    "inception4": _lazy("inception_model", "Inceptionv4Model"),
    "resnet50": _lazy("resnet_model", "create_resnet50_model"),
    "resnet50_v1.5": _lazy("resnet_model", "create_resnet50_v1_5_model"),
    "resnet50_v2": _lazy("resnet_model", "create_resnet50_v2_model"),
    "resnet101": _lazy("resnet_model", "create_resnet101_model"),
    "resnet101_v2": _lazy("resnet_model", "create_resnet101_v2_model"),
    "resnet152": _lazy("resnet_model", "create_resnet152_model"),
    "resnet152_v2": _lazy("resnet_model", "create_resnet152_v2_model"),
    "mobilenet": _lazy("mobilenet_v2", "MobilenetModel"),
    "nasnet": _lazy("nasnet_model", "NasnetModel"),
    "nasnetlarge": _lazy("nasnet_model", "NasnetLargeModel"),
    "ncf": _lazy("ncf_model", "NcfModel"),
}
for _d in (18, 34, 50, 101, 152, 200):
    _IMAGENET["official_resnet%d" % _d] = _lazy("official_resnet_model", "official_v1_%d" % _d)
    _IMAGENET["official_resnet%d_v2" % _d] = _lazy("official_resnet_model", "official_v2_%d" % _d)

_CIFAR = {
    "alexnet": _lazy("alexnet_model", "AlexnetCifar10Model"),
    "resnet20": _lazy("resnet_model", "create_resnet20_cifar_model"),
    "resnet20_v2": _lazy("resnet_model", "create_resnet20_v2_cifar_model"),
    "resnet32": _lazy("resnet_model", "create_resnet32_cifar_model"),
    "resnet32_v2": _lazy("resnet_model", "create_resnet32_v2_cifar_model"),
    "resnet44": _lazy("resnet_model", "create_resnet44_cifar_model"),
    "resnet44_v2": _lazy("resnet_model", "create_resnet44_v2_cifar_model"),
    "resnet56": _lazy("resnet_model", "create_resnet56_cifar_model"),
    "resnet56_v2": _lazy("resnet_model", "create_resnet56_v2_cifar_model"),
    "resnet110": _lazy("resnet_model", "create_resnet110_cifar_model"),
    "resnet110_v2": _lazy("resnet_model", "create_resnet110_v2_cifar_model"),
    "trivial": _lazy("trivial_model", "TrivialCifar10Model"),
    "densenet40_k12": _lazy("densenet_model", "create_densenet40_k12_model"),
    "densenet100_k12": _lazy("densenet_model", "create_densenet100_k12_model"),
    "densenet100_k24": _lazy("densenet_model", "create_densenet100_k24_model"),
    "nasnet": _lazy("nasnet_model", "NasnetCifarModel"),
}

_LIBRISPEECH = {"deepspeech2": _lazy("deepspeech", "DeepSpeech2Model")}
_COCO = {"ssd300": _lazy("ssd_model", "SSD300Model")}


def _get_model_map(dataset_name):
    if "cifar10" == dataset_name:
        return _CIFAR
    if dataset_name in ("imagenet", "synthetic"):
        return _IMAGENET
    if dataset_name == "librispeech":
        return _LIBRISPEECH
    if dataset_name == "coco":
        return _COCO
    raise ValueError("Invalid dataset name: %s" % dataset_name)


def get_model_config(model_name, dataset, params):
    model_map = _get_model_map(dataset.name)
    if model_name not in model_map:
        raise ValueError("Invalid model name '%s' for dataset '%s'" % (model_name, dataset.name))
    return model_map[model_name](params=params)


def register_model(model_name, dataset_name, model_func):
    model_map = _get_model_map(dataset_name)
    if model_name in model_map:
        raise ValueError("Model \"%s\" is already registered for dataset \"%s\""
                         % (model_name, dataset_name))
    model_map[model_name] = model_func


def list_models(dataset_name="imagenet"):
    return sorted(_get_model_map(dataset_name))
