"""Host-side transform construction, following pbrt-v4 util/transform.cpp.

Matrices are built in float64 and handed to the device (and to the oracle) as
row-major float32 4x4 — pbrt builds them in float; both the GPU path and the CPU
oracle consume the SAME float32 matrices, so parity between them is exact.
"""
import numpy as np


def translate(d):
    m = np.eye(4)
    m[:3, 3] = d
    return m


def scale(x, y, z):
    return np.diag([x, y, z, 1.0])


def rotate(theta_deg, axis):
    """transform.h:220-251 (Rodrigues form)."""
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    s, c = np.sin(np.radians(theta_deg)), np.cos(np.radians(theta_deg))
    m = np.eye(4)
    m[0, 0] = a[0] * a[0] + (1 - a[0] * a[0]) * c
    m[0, 1] = a[0] * a[1] * (1 - c) - a[2] * s
    m[0, 2] = a[0] * a[2] * (1 - c) + a[1] * s
    m[1, 0] = a[0] * a[1] * (1 - c) + a[2] * s
    m[1, 1] = a[1] * a[1] + (1 - a[1] * a[1]) * c
    m[1, 2] = a[1] * a[2] * (1 - c) - a[0] * s
    m[2, 0] = a[0] * a[2] * (1 - c) - a[1] * s
    m[2, 1] = a[1] * a[2] * (1 - c) + a[0] * s
    m[2, 2] = a[2] * a[2] + (1 - a[2] * a[2]) * c
    return m


def look_at(pos, look, up):
    """LookAt (transform.cpp:81-113): returns cameraFromWorld."""
    pos, look, up = (np.asarray(v, np.float64) for v in (pos, look, up))
    d = look - pos
    d = d / np.linalg.norm(d)
    upn = up / np.linalg.norm(up)
    right = np.cross(upn, d)
    if np.linalg.norm(right) == 0:
        raise ValueError("LookAt: up vector and viewing direction are parallel")
    right = right / np.linalg.norm(right)
    new_up = np.cross(d, right)
    world_from_camera = np.eye(4)
    world_from_camera[:3, 0] = right
    world_from_camera[:3, 1] = new_up
    world_from_camera[:3, 2] = d
    world_from_camera[:3, 3] = pos
    return np.linalg.inv(world_from_camera)


def orthographic(z_near, z_far):
    """transform.cpp:115-117."""
    return scale(1, 1, 1 / (z_far - z_near)) @ translate([0, 0, -z_near])


def perspective(fov_deg, n, f):
    """transform.cpp:119-131."""
    persp = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, f / (f - n), -f * n / (f - n)], [0, 0, 1, 0]],
                     dtype=np.float64)
    inv_tan = 1 / np.tan(np.radians(fov_deg) / 2)
    return scale(inv_tan, inv_tan, 1) @ persp


def f32(m):
    return np.ascontiguousarray(np.asarray(m, np.float64).astype(np.float32).reshape(4, 4))
