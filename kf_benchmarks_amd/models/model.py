"""Model base classes and the Network module that owns a model's variables.

``Model`` / ``CNNModel`` keep the reference's configuration API
(tcb/models/model.py:31-312): name, default batch size, learning rate, fp16
loss scale, input shapes/dtypes, synthetic inputs, build_network, loss and
accuracy functions.  Network construction is eager (see builder.py); the
model's variables live in a :class:`Network` ``nn.Module``.

Deliberate fix vs. the fork: the final affine (logits) layer is present
(the fork commented it out, tcb/models/model.py:269-272, so its "logits" were
the spatial mean and its loss was NaN).
"""

from __future__ import annotations

import collections
import re
from typing import List, Optional

import torch
from torch import nn

from ..ops import nn as F
from .builder import ConvNetBuilder
from .layers import AffineLayer, BatchNormLayer, ConvLayer, DepthwiseConvLayer, Layer

BuildNetworkResult = collections.namedtuple("BuildNetworkResult", ["logits", "extra_info"])


def _dtype_from_params(params):
    if params is None:
        return torch.float32
    if getattr(params, "use_fp16", False):
        return torch.float16
    if getattr(params, "use_bf16", False):
        return torch.bfloat16
    return torch.float32


class Model:
    """Base model configuration."""

    def __init__(self, model_name, batch_size, learning_rate, fp16_loss_scale, params=None):
        self.model_name = model_name
        self.batch_size = batch_size
        self.default_batch_size = batch_size
        self.learning_rate = learning_rate
        self.fp16_loss_scale = fp16_loss_scale
        self.params = params
        if params is not None:
            self.use_tf_layers = params.use_tf_layers
            self.fp16_vars = params.fp16_vars
        else:
            self.use_tf_layers = True
            self.fp16_vars = False
        self.data_type = _dtype_from_params(params)

    def get_model_name(self):
        return self.model_name

    def get_batch_size(self):
        return self.batch_size

    def set_batch_size(self, batch_size):
        self.batch_size = batch_size

    def get_default_batch_size(self):
        return self.default_batch_size

    def get_fp16_loss_scale(self):
        return self.fp16_loss_scale

    def custom_l2_loss(self, fp32_params):
        del fp32_params
        return None

    def l2_param_filter(self, scope_name: str) -> bool:
        """Variables included in the L2 loss (all trainable by default, as
        tcb/benchmark_cnn.py:3070-3099)."""
        return True

    def get_learning_rate(self, global_step, batch_size):
        del global_step, batch_size
        return self.learning_rate

    def get_input_shapes(self, subset):
        raise NotImplementedError

    def get_input_data_types(self, subset):
        raise NotImplementedError

    def get_synthetic_inputs(self, input_name, nclass, device="cpu", seed=0):
        raise NotImplementedError

    def build_network(self, inputs, phase_train, nclass):
        raise NotImplementedError

    def loss_function(self, inputs, build_network_result):
        raise NotImplementedError

    def accuracy_function(self, inputs, logits):
        raise NotImplementedError

    def postprocess(self, results):
        return results


class CNNModel(Model):
    """Base class for image CNNs built with the ConvNetBuilder."""

    def __init__(self, model, image_size, batch_size, learning_rate, layer_counts=None,
                 fp16_loss_scale=128, params=None):
        super().__init__(model, batch_size, learning_rate, fp16_loss_scale, params=params)
        self.image_size = image_size
        self.layer_counts = layer_counts
        self.depth = 3
        self.data_format = params.data_format if params is not None else "NCHW"

    def get_layer_counts(self):
        return self.layer_counts

    def skip_final_affine_layer(self):
        return False

    def add_inference(self, cnn):
        raise NotImplementedError

    def get_input_data_types(self, subset):
        del subset
        return [self.data_type, torch.int32]

    def get_input_shapes(self, subset):
        del subset
        # NHWC images and [batch] labels.
        return [[self.batch_size, self.image_size, self.image_size, self.depth],
                [self.batch_size]]

    def get_synthetic_inputs(self, input_name, nclass, device="cpu", seed=0):
        """Images ~ truncated normal(mean 127, std 60), labels ~ U[0, nclass-1)
        (tcb/models/model.py:220-237), generated on the target device."""
        del input_name
        image_shape, label_shape = self.get_input_shapes("train")
        images = F.synthetic_images(tuple(image_shape), self.data_type, device, seed)
        labels = F.synthetic_labels(label_shape[0], nclass, device, seed)
        return images, labels

    def build_network(self, inputs, phase_train=True, nclass=1001, network=None):
        if network is None:
            raise ValueError("build_network needs the Network that owns the variables")
        return network(inputs[0], phase_train=phase_train)

    def loss_function(self, inputs, build_network_result):
        _, labels = inputs
        loss = F.softmax_cross_entropy(build_network_result.logits, labels)
        aux = build_network_result.extra_info
        if aux is not None:
            loss = loss + 0.4 * F.softmax_cross_entropy(aux, labels)
        return loss

    def accuracy_function(self, inputs, logits):
        _, labels = inputs
        top1, top5 = F.in_top_k(logits, labels)
        return {"top_1_accuracy": top1, "top_5_accuracy": top5}


_SANITIZED = {}


def _sanitize(scope: str) -> str:
    # memoized: every forward looks up every layer by scope (host launch path)
    key = _SANITIZED.get(scope)
    if key is None:
        key = re.sub(r"[^0-9A-Za-z_]", lambda m: {"/": "__", ".": "_d_"}.get(m.group(0), "_"),
                     scope)
        _SANITIZED[scope] = key
    return key


class Network(nn.Module):
    """All variables of one model replica plus its eager forward.

    The first call (``materialize``) runs the model on a ``meta`` tensor of
    batch 1, which creates every layer; afterwards the set of layers is frozen
    and each forward looks them up by scope.
    """

    def __init__(self, model: CNNModel, nclass: int, device, compute_dtype=None,
                 kernel_impl: str = "hip", seed: int = 1234):
        super().__init__()
        self.model = model
        self.nclass = nclass
        self.param_device = torch.device(device)
        self.compute_dtype = compute_dtype or model.data_type
        self.kernel_impl = kernel_impl
        self.layers = nn.ModuleDict()
        self.scopes: List[str] = []
        self.init_gen = torch.Generator().manual_seed(seed)
        self._building = False
        self._dropout_seed = seed * 7919 + 17
        self.materialize()

    # -------------------------------------------------------------- layers
    def get_or_create(self, scope, factory) -> Layer:
        key = _sanitize(scope)
        if key in self.layers:
            return self.layers[key]
        if not self._building:
            raise KeyError("layer %s was not created during materialization" % scope)
        layer = factory()
        self.layers[key] = layer
        self.scopes.append(scope)
        return layer

    def next_dropout_seed(self, with_key=False):
        self._dropout_seed = (self._dropout_seed * 1103515245 + 12345) & 0x7FFFFFFF
        if not with_key:
            return self._dropout_seed
        # launch tape: the k-th dropout of the recorded step is the per-step
        # argument "dropout<k>" (tape_dropout_values re-derives them)
        k = getattr(self, "_dropout_calls", 0)
        self._dropout_calls = k + 1
        return self._dropout_seed, "dropout%d" % k

    def drop_path_kp(self, base, layer_ratio, total_steps, step=None):
        """NASNet drop-path keep probability of a cell at ``step`` (default:
        the current global step)."""
        kp = 1 - layer_ratio * (1 - base)
        step = float(getattr(self, "global_step", 0) if step is None else step)
        ratio = min(1.0, step / total_steps)
        return 1 - ratio * (1 - kp)

    def drop_path_key(self, base, layer_ratio, total_steps):
        """Per-step tape argument name of a drop-path keep probability (the
        schedule parameters are kept to re-derive it at every replay)."""
        if not hasattr(self, "_drop_paths"):
            self._drop_paths = {}
        spec = (base, layer_ratio, total_steps)
        for k, v in self._drop_paths.items():
            if v == spec:
                return k
        key = "droppath_kp_%d" % len(self._drop_paths)
        self._drop_paths[key] = spec
        return key

    def tape_begin_recording(self):
        self._dropout_calls = 0
        self._tape_dropouts = None

    def tape_end_recording(self):
        """Freezes the recorded step's dropout count: eager steps after the
        recording (accuracy / display steps) still advance _dropout_calls,
        but a replayed step holds exactly the recorded dropouts."""
        self._tape_dropouts = getattr(self, "_dropout_calls", 0)

    def tape_dropout_values(self):
        """The dropout seeds of the next replayed step: the generator
        advanced exactly as an eager step advances it."""
        out = {}
        for key, (base, ratio, total) in getattr(self, "_drop_paths", {}).items():
            # the step the replay trains (global_step is advanced after it)
            out[key] = self.drop_path_kp(base, ratio, total)
        n = getattr(self, "_tape_dropouts", None)
        for k in range(n if n is not None else getattr(self, "_dropout_calls", 0)):
            self._dropout_seed = (self._dropout_seed * 1103515245 + 12345) & 0x7FFFFFFF
            out["dropout%d" % k] = self._dropout_seed & 0xFFFFFFFF
        return out

    def materialize(self):
        shape = self.model.get_input_shapes("train")[0]
        images = torch.empty([1] + list(shape[1:]), dtype=self.compute_dtype, device="meta")
        self._building = True
        try:
            with torch.no_grad():
                self.forward(images, phase_train=True)
        finally:
            self._building = False

    # ------------------------------------------------------------- forward
    def forward_inputs(self, inputs, phase_train=True):
        """Engine entry: ``inputs`` is the tuple the input source yields
        (images, labels) for image models."""
        return self.forward(inputs[0], phase_train=phase_train)

    def forward(self, images, phase_train=True):
        model = self.model
        if phase_train and images.is_cuda:
            from ..ops.conv_hip import STATS_ARENA
            STATS_ARENA.reset(images.device)
        cnn = ConvNetBuilder(self, images, model.depth, phase_train, self.compute_dtype)
        model.add_inference(cnn)
        if model.skip_final_affine_layer():
            logits = cnn.top_layer
        else:
            logits = cnn.affine(self.nclass, activation="linear")
        aux_logits = None
        if cnn.aux_top_layer is not None:
            with cnn.switch_to_aux_top_layer():
                aux_logits = cnn.affine(self.nclass, activation="linear", stddev=0.001)
        return BuildNetworkResult(logits=logits, extra_info=aux_logits)

    # ----------------------------------------------------------- variables
    def ordered_layers(self):
        return [self.layers[_sanitize(s)] for s in self.scopes]

    def trainable_variables(self):
        """(tf_name, Parameter) in creation order."""
        out = []
        for layer in self.ordered_layers():
            for name, p in layer.named_parameters(recurse=False):
                out.append((layer.tf_scope + "/" + _tf_param_name(layer, name), p))
        return out

    def tf_variables(self, prefix="v0/cg/"):
        """{full TF name: tensor in TF layout} for checkpointing."""
        out = {}
        for layer in self.ordered_layers():
            for name, t in layer.tf_variables().items():
                out[prefix + layer.tf_scope + "/" + name] = t
        return out

    def load_tf_variables(self, values, prefix="v0/cg/", strict=True):
        loaded = 0
        for layer in self.ordered_layers():
            for name in layer.tf_variables().keys():
                full = prefix + layer.tf_scope + "/" + name
                if full in values:
                    layer.load_tf_variable(name, values[full])
                    loaded += 1
                elif strict:
                    raise KeyError("checkpoint is missing %s" % full)
        return loaded

    def num_params(self):
        return sum(p.numel() for _, p in self.trainable_variables())


class ModuleModel(Model):
    """Base for models that are not ConvNetBuilder image CNNs (NCF,
    DeepSpeech2, ...): the model supplies a torch module whose
    ``forward(inputs, phase_train)`` returns a BuildNetworkResult, and its own
    inputs, loss and accuracy (the reference's model.Model API,
    tcb/models/model.py:31-160)."""

    def make_module(self, nclass: int, device, dtype, gen: torch.Generator) -> nn.Module:
        raise NotImplementedError

    def accuracy_function(self, inputs, logits):
        return {}


class ModuleNetwork(nn.Module):
    """Network-compatible wrapper (trainable_variables / ordered_layers /
    tf_variables) around a ModuleModel's torch module."""

    def __init__(self, model: ModuleModel, nclass: int, device, compute_dtype=None,
                 kernel_impl: str = "hip", seed: int = 1234):
        super().__init__()
        self.model = model
        self.nclass = nclass
        self.param_device = torch.device(device)
        self.compute_dtype = compute_dtype or model.data_type
        self.kernel_impl = kernel_impl
        self.init_gen = torch.Generator().manual_seed(seed)
        self.body = model.make_module(nclass, self.param_device, self.compute_dtype,
                                      self.init_gen)

    def forward_inputs(self, inputs, phase_train=True):
        return self.body(inputs, phase_train)

    def forward(self, inputs, phase_train=True):
        return self.body(inputs, phase_train)

    # launch-tape hooks (Network's): the module models (DeepSpeech2, NCF)
    # draw no per-step dropout / drop-path values, so a replayed step has no
    # per-step network arguments
    def tape_begin_recording(self):
        pass

    def tape_end_recording(self):
        pass

    def tape_dropout_values(self):
        return {}

    def ordered_layers(self):
        return [m for m in self.body.modules()
                if any(True for _ in m.parameters(recurse=False))
                or any(True for _ in m.buffers(recurse=False))]

    def trainable_variables(self):
        return [(n.replace(".", "/"), p) for n, p in self.body.named_parameters()
                if p.requires_grad]

    def tf_variables(self, prefix="v0/cg/"):
        out = {prefix + n.replace(".", "/"): p.detach() for n, p in self.body.named_parameters()}
        for n, b in self.body.named_buffers():
            out[prefix + n.replace(".", "/")] = b
        return out

    def load_tf_variables(self, values, prefix="v0/cg/", strict=True):
        loaded = 0
        named = dict(self.body.named_parameters())
        named.update(dict(self.body.named_buffers()))
        for n, t in named.items():
            full = prefix + n.replace(".", "/")
            if full in values:
                with torch.no_grad():
                    t.copy_(torch.as_tensor(values[full], dtype=t.dtype).reshape(t.shape))
                loaded += 1
            elif strict:
                raise KeyError("checkpoint is missing %s" % full)
        return loaded

    def num_params(self):
        return sum(p.numel() for _, p in self.trainable_variables())


def make_network(model, nclass, device, compute_dtype=None, kernel_impl="hip", seed=1234):
    cls = ModuleNetwork if isinstance(model, ModuleModel) else Network
    return cls(model, nclass, device, compute_dtype, kernel_impl=kernel_impl, seed=seed)


def _tf_param_name(layer, attr):
    if isinstance(layer, DepthwiseConvLayer):
        return "depthwise_weights"
    if isinstance(layer, ConvLayer):
        return {"weight": "conv2d/kernel", "bias": "biases"}[attr]
    if isinstance(layer, AffineLayer):
        return attr
    if isinstance(layer, BatchNormLayer):
        return attr
    return attr
