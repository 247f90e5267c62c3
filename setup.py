"""Packaging: ``pip install -e .`` builds the in-tree gfx950 kernels + C++ runtime first.

The native libraries are written to ``rocket_amd/_lib`` (in-tree, next to the Python package),
which is where :mod:`rocket_amd.ops._lib` loads them from.
"""

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py
from setuptools.command.develop import develop


def _build_native():
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from rocket_amd.native import build

    build.build(force=False)


class BuildPy(build_py):
    def run(self):
        _build_native()
        super().run()


class Develop(develop):
    def run(self):
        _build_native()
        super().run()


setup(
    name="rocket_amd",
    version="0.1.0",
    description="MI355X-native training-loop engine with the capsule API of dsenushkin/rocket",
    packages=find_packages(include=["rocket_amd", "rocket_amd.*", "rocket", "rocket.*"]),
    package_data={"rocket_amd": ["_lib/*.so", "tuning/*.csv", "native/kernels/*.hip", "native/kernels/*.h", "native/runtime/*.cpp"]},
    python_requires=">=3.10",
    install_requires=["torch>=2.4", "numpy", "tqdm", "safetensors"],
    cmdclass={"build_py": BuildPy, "develop": Develop},
)
