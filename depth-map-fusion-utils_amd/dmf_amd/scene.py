"""Synthetic inputs for tests and the bench (SURVEY.md §8d "Synthetic inputs").

Input tooling, not part of the hot path: an analytic scene (sphere r=0.25 m at the
origin + a box standing on a ground plane z=-0.35 m), uint16-millimetre depth
frames rendered by ray/primitive intersection, per-pixel analytic normals, and
camera poses:

* ``fibonacci_poses`` — P cameras on a 0.7 m Fibonacci sphere looking at the
  origin (orthonormal, optional seeded jitter of +-5 mm / +-1 deg);
* ``reference_style_poses`` — the reference's own placement rule
  (include/Algorithms.hpp:190-236 positionCamera + :282-298 positionCameras):
  camera 300 mm along the surface normal with the x/y axes forced to
  (0,-1,0)/(1,0,0), i.e. NON-orthonormal 3x4 matrices, which exercise the general
  Affine3f inverse exactly like the reference drivers do.

Poses are float32 row-major 3x4 ``[R|t]`` camera->world (Eigen::Affine3f rows 0..2),
the convention of Camera::transformPoints (include/Camera.hpp:39-45).
"""
from __future__ import annotations

import numpy as np

# tests/Raytracing.cpp:61 — the reference intrinsics (640x480)
K_640x480 = np.array([602.39306640625, 0.0, 314.6370849609375,
                      0.0, 602.39306640625, 245.04962158203125,
                      0.0, 0.0, 1.0], np.float32)
# reference K x2 (1280x960), centre-cropped 120 rows -> 1280x720
K_1280x720 = np.array([1204.7861328125, 0.0, 629.274169921875,
                       0.0, 1204.7861328125, 370.0992431640625,
                       0.0, 0.0, 1.0], np.float32)

SPHERE_C = np.array([0.0, 0.0, 0.0])
SPHERE_R = 0.25
GROUND_Z = -0.35
BOX_LO = np.array([0.24, 0.24, -0.35])
BOX_HI = np.array([0.40, 0.40, -0.15])
DEPTH_MIN_MM = 200
DEPTH_MAX_MM = 1000  # exclusive (RayTracingEngine.hpp:24-25 k_ZMin/k_ZMax)


def intrinsics(width, height):
    if (width, height) == (640, 480):
        return K_640x480.copy()
    if (width, height) == (1280, 720):
        return K_1280x720.copy()
    raise ValueError(f"no intrinsics for {width}x{height}")


# ----------------------------------------------------------------------------- poses
def _rot(axis, ang):
    c, s = np.cos(ang), np.sin(ang)
    if axis == 0:
        return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])
    if axis == 1:
        return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def look_at(eye, target=(0.0, 0.0, 0.0)):
    """Camera->world rotation for x right, y down, z forward (Camera.hpp:24-31 frame)."""
    eye = np.asarray(eye, np.float64)
    f = np.asarray(target, np.float64) - eye
    f /= np.linalg.norm(f)
    up = np.array([0.0, 0.0, 1.0])
    if np.linalg.norm(np.cross(up, f)) < 1e-3:
        up = np.array([0.0, 1.0, 0.0])
    yd = -(up - np.dot(up, f) * f)
    yd /= np.linalg.norm(yd)
    xr = np.cross(yd, f)
    return np.stack([xr, yd, f], axis=1)


def fibonacci_poses(P, radius=0.7, seed=1234, jitter=True):
    """(P, 12) float32 poses on a Fibonacci sphere looking at the origin."""
    rng = np.random.default_rng(seed)
    golden = np.pi * (3.0 - np.sqrt(5.0))
    out = np.zeros((P, 12), np.float32)
    for i in range(P):
        z = 1.0 - 2.0 * (i + 0.5) / P
        rr = np.sqrt(max(0.0, 1.0 - z * z))
        phi = i * golden
        eye = radius * np.array([rr * np.cos(phi), rr * np.sin(phi), z])
        R = look_at(eye)
        if jitter:
            eye = eye + rng.uniform(-0.005, 0.005, 3)
            a = np.deg2rad(rng.uniform(-1.0, 1.0, 3))
            R = R @ _rot(0, a[0]) @ _rot(1, a[1]) @ _rot(2, a[2])
        M = np.concatenate([R, eye[:, None]], axis=1)
        out[i] = M.astype(np.float32).reshape(12)
    return out


def reference_style_poses(points, normals, distance_mm=300):
    """include/Algorithms.hpp:282-298 positionCameras -> :190-236 positionCamera.

    Flip normals with n_z <= 0, camera centre = movePointAway(p, n, d/1000)
    (Algorithms.hpp:114-122, float n*d then + double p), z axis = -n, x/y axes
    forced to (0,-1,0) / (1,0,0) (:225-226).
    """
    points = np.asarray(points, np.float32).reshape(-1, 3)
    normals = np.asarray(normals, np.float32).reshape(-1, 3).copy()
    out = np.zeros((points.shape[0], 12), np.float32)
    dist = np.float32(np.float64(distance_mm) / 1000.0)
    for i in range(points.shape[0]):
        n = normals[i].copy()
        if n[2] <= 0:
            n = -n
        nor = (-n).astype(np.float32)
        moved = (n * dist).astype(np.float32).astype(np.float64) + points[i].astype(np.float64)
        Q = np.zeros((3, 4), np.float32)
        Q[:, 0] = (0.0, -1.0, 0.0)
        Q[:, 1] = (1.0, 0.0, 0.0)
        Q[:, 2] = nor
        Q[:, 3] = moved.astype(np.float32)
        out[i] = Q.reshape(12)
    return out


def write_pose_file(path, poses):
    """include/FileRoutines.hpp:98-112 writeCameraLocations format (N, then 3 CSV rows/pose)."""
    poses = np.asarray(poses, np.float32).reshape(-1, 3, 4)
    with open(path, "w") as f:
        f.write(f"{poses.shape[0]}\n")
        for M in poses:
            for j in range(3):
                f.write(",".join(repr(float(v)) for v in M[j]) + "\n")


def read_pose_file(path):
    """include/FileRoutines.hpp:69-96 readCameraLocations (stof per field)."""
    with open(path) as f:
        n = int(f.readline())
        out = np.zeros((n, 12), np.float32)
        for i in range(n):
            rows = [f.readline().strip().split(",") for _ in range(3)]
            out[i] = np.array([float(v) for r in rows for v in r], np.float32)
    return out


# ----------------------------------------------------------------------------- render
def render(K, width, height, pose, dmin=DEPTH_MIN_MM, dmax=DEPTH_MAX_MM):
    """Render one frame -> (depth uint16 [H,W] mm, normals float32 [H,W,3] world).

    Depth is the camera-z distance (Camera.hpp:24-31 scales x,y by z), quantised
    to whole millimetres; pixels with no hit or outside [dmin, dmax) are 0.
    """
    K = np.asarray(K, np.float64)
    fx, cx, fy, cy = K[0], K[2], K[4], K[5]
    M = np.asarray(pose, np.float64).reshape(3, 4)
    R, o = M[:, :3], M[:, 3]
    rr, cc = np.meshgrid(np.arange(height, dtype=np.float64), np.arange(width, dtype=np.float64), indexing="ij")
    dc = np.stack([(cc - cx) / fx, (rr - cy) / fy, np.ones_like(cc)], axis=-1)
    d = dc @ R.T  # world direction with camera-z component 1
    best = np.full(rr.shape, np.inf)
    nrm = np.zeros(rr.shape + (3,))
    # sphere
    oc = o - SPHERE_C
    a = np.einsum("ijk,ijk->ij", d, d)
    b = 2.0 * (d @ oc)
    c = oc @ oc - SPHERE_R ** 2
    disc = b * b - 4 * a * c
    ok = disc >= 0
    sq = np.sqrt(np.where(ok, disc, 0.0))
    s1 = (-b - sq) / (2 * a)
    s2 = (-b + sq) / (2 * a)
    s = np.where(s1 > 1e-6, s1, s2)
    hit = ok & (s > 1e-6) & (s < best)
    best = np.where(hit, s, best)
    p = o + d * s[..., None]
    nrm = np.where(hit[..., None], (p - SPHERE_C) / SPHERE_R, nrm)
    # ground plane z = GROUND_Z (two-sided)
    with np.errstate(divide="ignore", invalid="ignore"):
        sp = (GROUND_Z - o[2]) / d[..., 2]
    hit = np.isfinite(sp) & (sp > 1e-6) & (sp < best)
    best = np.where(hit, sp, best)
    pn = np.array([0.0, 0.0, 1.0 if o[2] >= GROUND_Z else -1.0])
    nrm = np.where(hit[..., None], pn, nrm)
    # box (slabs)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t0 = (BOX_LO - o) * inv
        t1 = (BOX_HI - o) * inv
    tmin = np.minimum(t0, t1)
    tmax = np.maximum(t0, t1)
    tmin = np.where(np.isnan(tmin), -np.inf, tmin)
    tmax = np.where(np.isnan(tmax), np.inf, tmax)
    tn = tmin.max(axis=-1)
    tf = tmax.min(axis=-1)
    hit = (tn <= tf) & (tn > 1e-6) & (tn < best)
    best = np.where(hit, tn, best)
    ax = tmin.argmax(axis=-1)
    bn = np.zeros(rr.shape + (3,))
    sgn = -np.sign(np.take_along_axis(d, ax[..., None], axis=-1)[..., 0])
    np.put_along_axis(bn, ax[..., None], sgn[..., None], axis=-1)
    nrm = np.where(hit[..., None], bn, nrm)
    mm = np.where(np.isfinite(best), np.round(best * 1000.0), 0.0)
    valid = (mm >= dmin) & (mm < dmax)
    depth = np.where(valid, mm, 0).astype(np.uint16)
    nrm = np.where(valid[..., None], nrm, 0.0).astype(np.float32)
    return depth, nrm


def render_frames(K, width, height, poses, dmin=DEPTH_MIN_MM, dmax=DEPTH_MAX_MM, normals=False, threads=None):
    """Render P frames; frames are independent, so they render on a thread pool (numpy
    releases the GIL in the per-frame array work).  threads=None: the job's CPU share
    (OMP_NUM_THREADS, else os.cpu_count(), at most 16)."""
    import os
    from concurrent.futures import ThreadPoolExecutor
    poses = np.asarray(poses, np.float32).reshape(-1, 12)
    P = poses.shape[0]
    depth = np.zeros((P, height, width), np.uint16)
    nrm = np.zeros((P, height, width, 3), np.float32) if normals else None
    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(int(threads), 16, P))

    def one(i):
        dd, nn = render(K, width, height, poses[i], dmin, dmax)
        depth[i] = dd
        if normals:
            nrm[i] = nn
    if threads == 1:
        for i in range(P):
            one(i)
    else:
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(one, range(P)))
    return (depth, nrm) if normals else depth


def grid_bounds(n):
    """bounds [-0.5, 0.5]^3 with n cells per axis (exact binary deltas)."""
    return (-0.5, 0.5, -0.5, 0.5, -0.5, 0.5), (n, n, n)


def sphere_centres(V=1024, radius=0.45, seed=11):
    """(V, 12) float32 identity-rotation poses whose centres lie on a `radius` sphere inside
    the volume (the createCameraLocationsFromSphere layout the run_tsp cost map is built over,
    tests/CameraPathGen.cpp:310-331): bench.py's collision cost map workload."""
    rng = np.random.default_rng(seed)
    dirs = rng.normal(size=(V, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    cp = np.tile(np.eye(3, 4, dtype=np.float32).reshape(1, 12), (V, 1))
    cp[:, 3::4] = (radius * dirs).astype(np.float32)
    return cp
