"""Packaging hook: the native module is built by ``akka_allreduce_amd._build``
(g++ for host code, hipcc --offload-arch=gfx950 for the kernels, linked against
the HIP runtime and RCCL inside the installed torch) before the Python files
are collected, so ``pip install -e .`` and wheels carry the same in-tree .so
that ``python -c "import __graft_entry__ as g; g.build()"`` produces."""
import os
import sys

from setuptools import setup
from setuptools.command.build_py import build_py


class BuildNative(build_py):
    def run(self):
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from akka_allreduce_amd._build import build

        build()
        super().run()


setup(cmdclass={"build_py": BuildNative})
