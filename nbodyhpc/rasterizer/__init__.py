"""Drop-in import path ``nbodyhpc.rasterizer`` (the reference's module name,
rasterization/src/python/nbodyhpc/rasterizer/__init__.py) served by the HIP
deposit kernel."""
from nbodyhpc_amd.rasterizer import (  # noqa: F401
    DeviceContainer, PointRenderer, VulkanContainer, get_default_container, get_point_renderer,
    render_knn_volume, render_points, render_points_volume)

__all__ = ["DeviceContainer", "PointRenderer", "VulkanContainer", "get_default_container",
           "get_point_renderer", "render_knn_volume", "render_points", "render_points_volume"]
