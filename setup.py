"""setuptools shim: compile the native components in-tree before packaging them.

``pip install .`` (or ``python setup.py build``) runs
``k8s_gpu_node_checker_amd.build`` so the wheel ships ``_native/*.so``;
the HIP library needs ``hipcc`` (ROCm) and is skipped, with a message, on
hosts without it.
"""
import os
import sys

from setuptools import setup
from setuptools.command.build_py import build_py

HERE = os.path.dirname(os.path.abspath(__file__))


class BuildNative(build_py):
    def run(self):
        sys.path.insert(0, HERE)
        from k8s_gpu_node_checker_amd.build import build
        for msg in build():
            print(msg)
        super().run()


setup(cmdclass={"build_py": BuildNative})
