"""Drop-in import path ``nbodyhpc.kdtree`` (the reference's module name,
kdtree/src/python/nbodyhpc/kdtree/__init__.py) served by the MI355X build."""
from nbodyhpc_amd.kdtree import KDTree, cKDTree, device_count  # noqa: F401
from nbodyhpc_amd.kdtree import _impl  # noqa: F401

__all__ = ["KDTree", "cKDTree", "device_count"]
