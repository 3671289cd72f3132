#!/usr/bin/env python3
"""Drop-in replacement for the reference's ``check-gpu-node.py`` entry point.

``python check-gpu-node.py [flags]`` behaves like the reference script
(same flags, output, exit codes); the implementation lives in the
``k8s_gpu_node_checker_amd`` package next to this file.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from k8s_gpu_node_checker_amd.cli import entry  # noqa: E402

if __name__ == "__main__":
    entry()
