"""Keras-style micro-benchmarks (role of the reference's keras_benchmarks/:
mnist_mlp, cifar10_cnn and lstm trained with ``fit`` for 2 epochs on random
data, timed per epoch).  A small Sequential / fit API over torch modules
replaces Keras; metrics go to a JSON-lines file instead of BigQuery."""
