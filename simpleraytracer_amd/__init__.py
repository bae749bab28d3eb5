"""simpleraytracer_amd -- MI355X-native brute-force primary-ray renderer behind the
ml* C ABI of the reference's libModelRunner.so.

Layers:
  csrc/        HIP kernels (render.hip) + C++ host objects (Context/Image/Model/Renderer)
  _native.py   ctypes binding of lib/libModelRunner.so
  runner.py    Python mirror of the ml* API (Context, Model, Image, render())
  device.py    scene files + device-level stages on caller buffers (DeviceScene)
  bands.py     row-band partition and the one-process-per-GPU band gather
"""
from .device import (MAX_BATCH, DeviceScene, SrtError, convert_scene, read_scene, scene_frame,  # noqa: F401
                     scene_triangles, write_scene)
from .runner import Context, Image, MLError, Model, default_offsets, render  # noqa: F401

__all__ = [
    "Context", "Image", "Model", "MLError", "render", "default_offsets",
    "DeviceScene", "SrtError", "MAX_BATCH", "write_scene", "scene_triangles", "scene_frame", "read_scene", "convert_scene",
]
