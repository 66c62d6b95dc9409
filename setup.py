"""setuptools shim: ``pip install .`` / ``python setup.py build_ext --inplace`` compile the gfx950
extension with the package's own build driver (hipcc for csrc/*.hip, the host compiler for
csrc/*.cpp, linked against the HIP runtime and RCCL bundled with torch; see _build.py)."""
from setuptools import setup
from setuptools.command.build_py import build_py
from setuptools.command.build_ext import build_ext


class _NativeBuild(build_ext):
    def run(self):
        from tutorial_torch_distributed_data_parallel_amd import _build

        _build.build()


class _BuildPy(build_py):
    def run(self):
        self.run_command("build_ext")
        super().run()


setup(cmdclass={"build_ext": _NativeBuild, "build_py": _BuildPy})
