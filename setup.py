"""Installs mythril_amd as a Mythril plugin (the drop-in of SURVEY.md §8b).

The reference finds external plugins only through the setuptools entry-point group
``mythril.plugins`` (mythril/plugin/discovery.py:17-21) and loads the default-enabled ones when
the CLI module is imported (mythril/interfaces/cli.py:39, plugin/loader.py:73-80).  Installing
this package next to mythril is therefore the whole integration step:

    make -C mythril_amd/csrc          # libmythril_hip.so for gfx950 (or let build_py run it)
    pip install .                     # entry point constraint-sieve -> SievePluginBuilder

``MYTHRIL_AMD_SIEVE=0`` disables the plugin without uninstalling it.
"""
import os
import subprocess

from setuptools import setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(ROOT, "mythril_amd", "libmythril_hip.so")


class BuildWithLibrary(build_py):
    """Builds libmythril_hip.so (hipcc, gfx950) before the package files are collected."""

    def run(self):
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", os.path.join(ROOT, "mythril_amd", "csrc")], check=True)
        super().run()


setup(
    name="mythril-amd",
    version="0.2.0",
    description="MI355X constraint sieve for Mythril's LASER engine (get_model front end)",
    packages=["mythril_amd"],
    package_data={"mythril_amd": ["libmythril_hip.so", "synth_spec.json"]},
    python_requires=">=3.8",
    install_requires=["numpy"],
    entry_points={
        "mythril.plugins": ["constraint-sieve = mythril_amd.plugin:SievePluginBuilder"],
    },
    cmdclass={"build_py": BuildWithLibrary},
)
