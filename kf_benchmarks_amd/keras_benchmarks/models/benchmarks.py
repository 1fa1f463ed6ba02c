"""The three Keras micro-benchmarks (roles of keras_benchmarks/models/
mnist_mlp_benchmark.py, cifar10_cnn_benchmark.py, lstm_benchmark.py):
2 epochs over 1000 random samples; ``total_time`` sums the epochs after the
first (the first includes graph/kernel warm-up)."""

from __future__ import annotations

import numpy as np

from .. import data_generator as dg
from ..sequential import (LSTM, Conv2D, Dense, Dropout, Flatten, MaxPooling2D, RMSprop,
                          Sequential, TimeHistory)


class _Bench:
    test_name = ""
    sample_type = "images"
    batch_size = 32
    epochs = 2
    num_samples = 1000

    def __init__(self):
        self.total_time = 0.0

    def _finish(self, cb):
        self.total_time = float(sum(cb.times[1:]))
        return self.total_time


class MnistMlpBenchmark(_Bench):
    test_name, sample_type, batch_size = "mnist_mlp", "images", 128

    def run_benchmark(self, gpus=0, device=None):
        x, y = dg.generate_img_input_data((self.num_samples, 28, 28))
        x = x.reshape(self.num_samples, 784).astype("float32") / 255
        y = dg.to_categorical(y, 10)
        m = Sequential(device)
        m.add(Dense(512, activation="relu", input_shape=(784,)))
        m.add(Dropout(0.2))
        m.add(Dense(512, activation="relu"))
        m.add(Dropout(0.2))
        m.add(Dense(10, activation="softmax"))
        m.compile(optimizer=RMSprop(), metrics=["accuracy"])
        cb = TimeHistory()
        m.fit(x, y, batch_size=self.batch_size, epochs=self.epochs, callbacks=[cb])
        return self._finish(cb)


class Cifar10CnnBenchmark(_Bench):
    test_name, sample_type, batch_size = "cifar10_cnn", "images", 32

    def run_benchmark(self, gpus=0, device=None):
        x, y = dg.generate_img_input_data((self.num_samples, 3, 32, 32))
        x = x.transpose(0, 2, 3, 1).astype("float32") / 255  # channels_last
        y = dg.to_categorical(y, 10)
        m = Sequential(device)
        m.add(Conv2D(32, (3, 3), padding="same", input_shape=x.shape[1:], activation="relu"))
        m.add(Conv2D(32, (3, 3), activation="relu"))
        m.add(MaxPooling2D((2, 2)))
        m.add(Dropout(0.25))
        m.add(Conv2D(64, (3, 3), padding="same", activation="relu"))
        m.add(Conv2D(64, (3, 3), activation="relu"))
        m.add(MaxPooling2D((2, 2)))
        m.add(Dropout(0.25))
        m.add(Flatten())
        m.add(Dense(512, activation="relu"))
        m.add(Dropout(0.5))
        m.add(Dense(10, activation="softmax"))
        m.compile(optimizer=RMSprop(lr=0.0001, decay=1e-6), metrics=["accuracy"])
        cb = TimeHistory()
        m.fit(x, y, batch_size=self.batch_size, epochs=self.epochs, shuffle=True, callbacks=[cb])
        return self._finish(cb)


class LstmBenchmark(_Bench):
    test_name, sample_type, batch_size = "lstm", "text", 128

    def run_benchmark(self, gpus=0, device=None):
        x, y = dg.generate_text_input_data((self.num_samples, 40, 60))
        m = Sequential(device)
        m.add(LSTM(128, input_shape=(40, 60)))
        m.add(Dense(60), activation="softmax")
        m.compile(optimizer=RMSprop(lr=0.01))
        cb = TimeHistory()
        m.fit(x.astype(np.float32), y.astype(np.float32), batch_size=self.batch_size,
              epochs=self.epochs, callbacks=[cb])
        return self._finish(cb)
