"""Import alias for the package directory ``assignment--2-group7-distributed-k-means_amd/``
(whose name is not a Python identifier): ``import kmeans_amd`` returns that package,
registered under the name ``kmeans_amd`` (submodules: ``kmeans_amd.engine`` ...)."""
import importlib.util
import os
import sys

_PKG = "assignment--2-group7-distributed-k-means_amd"
_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), _PKG)

_spec = importlib.util.spec_from_file_location(__name__, os.path.join(_DIR, "__init__.py"),
                                               submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
