#!/usr/bin/env python3
"""Drop-in CLI: same flags as tf_cnn_benchmarks.py (see kf_benchmarks_amd/params.py)."""
import sys

from kf_benchmarks_amd.cli import main

if __name__ == "__main__":
    sys.exit(main())
