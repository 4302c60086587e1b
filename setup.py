"""Packaging with the native build hooked in: ``pip install .`` compiles every
``csrc/*.hip`` kernel for gfx950 with hipcc (``distributed_ml_pytorch_amd/_build.py``)
before the package files are collected, so the wheel carries ``_native*.so``."""
from setuptools import setup
from setuptools.command.build_py import build_py


class BuildWithNative(build_py):
    def run(self):
        from distributed_ml_pytorch_amd import _build

        _build.build(verbose=True)
        super().run()


setup(cmdclass={"build_py": BuildWithNative})
