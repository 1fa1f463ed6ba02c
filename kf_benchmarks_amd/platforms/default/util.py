"""Default platform (role of tcb/platforms/default/util.py): cluster
manager, python-module command lines, test directories, one-time init."""

from __future__ import annotations

import os
import sys
import tempfile

from ... import cnn_util

_ROOT_PROJECT_DIR = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(cnn_util.__file__))))
_PACKAGE_DIR = os.path.dirname(os.path.abspath(cnn_util.__file__))

__all__ = ["define_platform_params", "get_cluster_manager", "get_command_to_run_python_module",
           "get_test_output_dir", "get_test_data_dir", "initialize"]


def define_platform_params():
    """No platform-specific flags on the default platform."""


def get_cluster_manager(params, config_proto=None):
    return cnn_util.TorchClusterManager(params, config_proto)


def get_command_to_run_python_module(module):
    if not sys.executable:
        raise ValueError("Could not find Python interpreter")
    return [sys.executable, "-m", "kf_benchmarks_amd." + module]


def get_test_output_dir():
    base = os.environ.get("TEST_OUTPUTS_DIR", os.path.join(tempfile.gettempdir(),
                                                           "kf_benchmarks_test_outputs"))
    os.makedirs(base, exist_ok=True)
    return tempfile.mkdtemp(dir=base)


def get_test_data_dir():
    """Generated fixtures live under the test output dir; the package's
    generator (data/test_data.py) writes them on demand."""
    d = os.environ.get("KFB_TEST_DATA_DIR", os.path.join(tempfile.gettempdir(),
                                                         "kf_benchmarks_test_data"))
    if not os.path.isdir(os.path.join(d, "fake_tf_record_data")):
        from ...data import test_data
        test_data.write_black_and_white_tfrecord_data(os.path.join(d, "fake_tf_record_data"),
                                                      num_classes=10)
    return d


_is_initialized = False


def initialize(params, config_proto=None):
    global _is_initialized
    if _is_initialized:
        return
    _is_initialized = True
    del params, config_proto
