"""Packaging: all metadata lives here so every setuptools in use builds the same distribution.

Ubuntu 22.04 (the ROCm image and this container) ships setuptools 59.6, which
predates PEP 621 and ignores a ``[project]`` table: metadata kept only in
``pyproject.toml`` built an empty ``UNKNOWN-0.0.0``.  So name, version,
packages, package data, entry points and dependencies are spelled out below,
and ``pyproject.toml`` carries only the build-system and pytest tables.

Offline there is no index to fetch a build backend from, so install with::

    pip install --no-build-isolation .

``build_py`` first runs ``k8s_gpu_node_checker_amd.build`` so the wheel ships
``_native/*.so`` and the ``mi355x-probe`` CLI; the HIP libraries need
``hipcc`` (ROCm) and are skipped, with a message, on hosts without it.
Reference packaging for comparison: ``/root/reference/pyproject.toml:1-11``
(a virtual uv project with no entry point, run as ``python check-gpu-node.py``).
"""
import os
import re
import sys

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = "k8s_gpu_node_checker_amd"


def _version() -> str:
    with open(os.path.join(HERE, PKG, "__init__.py"), encoding="utf-8") as f:
        m = re.search(r'^__version__ = "([^"]+)"', f.read(), re.M)
    if not m:
        raise RuntimeError("no __version__ in the package")
    return m.group(1)


class BuildNative(build_py):
    """Compile the native components in-tree, then copy them like any other package data."""

    def run(self):
        # K8SGNC_NATIVE_PREBUILT=1: package the _native/ already in the tree as is (the install test
        # copies a built tree; its .cmd stamps name the original paths and would force a rebuild)
        if os.environ.get("K8SGNC_NATIVE_PREBUILT") != "1":
            sys.path.insert(0, HERE)
            from k8s_gpu_node_checker_amd.build import build
            for msg in build():
                print(msg)
        super().run()


# setuptools 59.6 has no recursive ``**`` in package_data: one pattern per depth
PACKAGE_DATA = [
    "_native/*",
    "csrc/*/*.cpp", "csrc/*/*.h", "csrc/*/*.hip",
]

setup(
    name="k8s-gpu-node-checker-amd",
    version=_version(),
    description="MI355X-native Kubernetes GPU-node checker: same CLI/JSON/exit codes/Slack as "
                "k8s-gpu-node-checker, plus amd-smi + HIP health gating",
    long_description=open(os.path.join(HERE, "README.md"), encoding="utf-8").read(),
    long_description_content_type="text/markdown",
    license="MIT",
    python_requires=">=3.10",
    packages=find_packages(HERE, include=[PKG, PKG + ".*"]),
    package_data={PKG: PACKAGE_DATA},
    include_package_data=False,
    zip_safe=False,
    # Runtime is stdlib-only on the check path; PyYAML reads YAML kubeconfigs (miniyaml is the fallback).
    install_requires=["PyYAML>=5.4"],
    extras_require={
        # torch (ROCm) is only needed for the RCCL/xGMI collective diagnostic and bench.py's multi-GPU mode
        "collectives": ["torch"],
        # the node agent's kubelet PodResources client (kube/podresources.py: GPUs allocated to pods)
        "agent": ["grpcio"],
        "test": ["pytest", "hypothesis", "requests"],
    },
    entry_points={
        "console_scripts": [
            "check-gpu-node = k8s_gpu_node_checker_amd.cli:entry",
            # kubectl plugin: `kubectl gpu-node-checker --mi355x`, `kubectl gpu-node-checker --explain NODE`
            "kubectl-gpu_node_checker = k8s_gpu_node_checker_amd.cli:entry",
            "k8s-gpu-node-agent = k8s_gpu_node_checker_amd.agent.agent:main",
            "mi355x-diag = k8s_gpu_node_checker_amd.ops.diag:main",
            "mi355x-fabric = k8s_gpu_node_checker_amd.ops.fabric:main",
        ],
    },
    cmdclass={"build_py": BuildNative},
)
