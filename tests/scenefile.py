"""Write scene files (DESIGN.md "Scene file") from numpy arrays, for hand-built test scenes."""
from __future__ import annotations

import struct

import numpy as np

HEADER = struct.Struct("<8sIIQ10f3ff")  # 80 bytes


def write_custom_scene(path, vertices, albedo=None, eye=(0, 0, 0), lookat=(0, 0, 1), up=(0, 1, 0), vfov=60.0,
                       background=(0.0, 0.0, 0.0)):
    v = np.ascontiguousarray(np.asarray(vertices, np.float32).reshape(-1, 9))
    n = v.shape[0]
    a = np.full((n, 3), 0.5, np.float32) if albedo is None else np.asarray(albedo, np.float32).reshape(n, 3)
    with open(path, "wb") as f:
        f.write(HEADER.pack(b"SRTSCN01", 1, 0, n, *eye, *lookat, *up, vfov, *background, 0.0))
        f.write(v.tobytes())
        f.write(np.ascontiguousarray(a).tobytes())
    return str(path)


def read_scene(path):
    with open(path, "rb") as f:
        head = HEADER.unpack(f.read(HEADER.size))
        n = head[3]
        v = np.frombuffer(f.read(n * 36), np.float32).reshape(n, 9)
        a = np.frombuffer(f.read(n * 12), np.float32).reshape(n, 3)
    cam = np.array(head[4:14], np.float32)
    bg = np.array(head[14:17], np.float32)
    return cam, bg, v, a
