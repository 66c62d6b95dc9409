#!/usr/bin/env python3
"""Thin wrapper: see tutorial_torch_distributed_data_parallel_amd/cli.py::train_ddp."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tutorial_torch_distributed_data_parallel_amd.cli import train_ddp  # noqa: E402

if __name__ == "__main__":
    sys.exit(train_ddp())
