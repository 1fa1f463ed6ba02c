"""Random training data (role of keras_benchmarks/data_generator.py)."""

import numpy as np


def generate_img_input_data(input_shape, num_classes=10, seed=0):
    """(x_train int in [0, 255) of ``input_shape``, y_train in [0, num_classes))."""
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 255, input_shape)
    y = rng.integers(0, num_classes, (input_shape[0],))
    return x, y


def generate_text_input_data(input_shape, p=0.05, return_as_bool=True, seed=0):
    """One-hot-ish token presence: x [n, t, v], y [n, v] ~ Bernoulli(p)."""
    rng = np.random.default_rng(seed)
    x = rng.binomial(1, p, input_shape)
    y = rng.binomial(1, p, (input_shape[0], input_shape[2]))
    if return_as_bool:
        return x.astype(bool), y.astype(bool)
    return x, y


def to_categorical(y, num_classes):
    out = np.zeros((len(y), num_classes), np.float32)
    out[np.arange(len(y)), np.asarray(y).reshape(-1)] = 1.0
    return out
