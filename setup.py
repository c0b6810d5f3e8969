"""Install metadata (reference: setup.py:16-40, requirements.txt:1-26).

The reference's setup.py declares a pure-Python package with optional
``xgboost`` / ``keras`` extras. Here the GBDT engine and the Genetic-CNN
kernels are native code of this repository, so there are no model extras:
``build_py`` first compiles ``gentun_amd/_native/*.so`` in-tree
(g++ for the host GBDT engine, ``hipcc --offload-arch=gfx950`` for the HIP
kernels; ``GENTUN_HIP_ARCH`` overrides the target) and ships them as package
data. ``pip install -e .`` / ``python setup.py develop`` keep the in-tree
libraries that ``tools/build_native.py`` builds.

Both import names are installed: ``gentun_amd`` and the API-compatible
``gentun`` alias (reference module paths ``gentun.master``,
``gentun.models.keras_models`` ... resolve to the MI355X implementations).
"""

import os
import sys

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


class BuildNativeThenPy(build_py):
    """Compile the native libraries before the Python files are copied."""

    def run(self):
        sys.path.insert(0, ROOT)
        from tools import build_native
        build_native.build_all(verbose=True)
        super().run()


setup(
    name="gentun-amd",
    version="0.1.0",
    description="MI355X-native distributed genetic-algorithm search (Genetic-CNN + GBDT individuals), "
                "gentun-compatible API",
    long_description=open(os.path.join(ROOT, "README.md")).read(),
    long_description_content_type="text/markdown",
    license="Apache-2.0",
    python_requires=">=3.9",
    packages=find_packages(include=["gentun_amd", "gentun_amd.*", "gentun", "gentun.*"]),
    package_data={"gentun_amd": ["_native/*.so"]},
    install_requires=["numpy", "torch"],
    extras_require={
        # data helpers of the example drivers (reference extras: setup.py:35-39)
        "examples": ["pandas", "scikit-learn"],
        "test": ["pytest", "pytest-timeout", "scikit-learn"],
    },
    entry_points={"console_scripts": ["gentun-amd = gentun_amd.__main__:main"]},
    cmdclass={"build_py": BuildNativeThenPy},
)
