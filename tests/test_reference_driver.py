"""The reference's own drivers tests/Raytracing.cpp (:55-105) and tests/SetCover.cpp
(:218-330), compiled UNCHANGED from /root/reference against the drop-in headers (depth-map-fusion-utils_amd/
compat first on the include path; headless PCL/Eigen/Boost stand-ins for the I/O,
downsampling and viewer calls it makes around the hot path) and linked to libdmf.so.

* CPU: the file compiles and links as is (where the reference checkout exists; the
  binary built by __graft_entry__.build() travels with the tree to the GPU box).
* GPU: the binary runs headless on a synthetic PCD (ASCII and binary): readPointCloud ->
  getMinMax3D -> VoxelVolume setup + integratePointCloud -> downsample + positionCameras
  -> reverseRayTraceFast(camera 0, viz) -> addVolumeWithVoxelsClassified, whose dump is
  checked against the oracle running the same sequence: volume geometry, occupied_cells_
  order, the camera pose (against a numpy restatement of VoxelGrid + positionCameras) and
  every voxel's view / good flag;
* GPU: SetCover.cpp runs headless (its viewer thread ends at once, its input thread runs the
  pipeline): positionCameras(downsample(cloud, 0.1), 500) filtered to z >= 0, the
  reverseRayTraceFast good set of every camera, greedySetCover, and writeCameraLocations
  of the selected cameras, which must equal the oracle's selection of the same cameras.
"""
import os
import subprocess

import numpy as np
import pytest

import helpers as Hh
from dmf_amd import scene

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "depth-map-fusion-utils_amd")
REF_SRC = "/root/reference/tests/Raytracing.cpp"
REF_SC = "/root/reference/tests/SetCover.cpp"
BINARY = os.path.join(PKG, "build", "raytracing_ref")
BINARY_SC = os.path.join(PKG, "build", "setcover_ref")
K_REF = np.array([602.39306640625, 0.0, 314.6370849609375, 0.0, 602.39306640625, 245.04962158203125, 0.0, 0.0, 1.0],
                 np.float32).reshape(3, 3)  # Raytracing.cpp:61


@pytest.mark.skipif(not os.path.isfile(REF_SRC), reason="reference checkout absent")
@pytest.mark.parametrize("src", [REF_SRC, REF_SC])
def test_reference_drivers_compile_unchanged(tmp_path, src):
    exe = tmp_path / "driver"
    r = subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(PKG, "compat"), "-I",
                        os.path.join(PKG, "compat", "shims"), "-I", os.path.join(ROOT, "include"),
                        src, "-o", str(exe), "-L", os.path.join(PKG, "build"), "-ldmf", "-lpthread"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    syms = subprocess.run(["nm", "-u", str(exe)], capture_output=True, text=True, check=True).stdout
    for s in ("dmf_volume_create", "dmf_volume_integrate", "dmf_reverse_ray_trace_fast"):
        assert s in syms, s  # the hot path goes through libdmf.so
    # the reference sources are compiled in place, never copied into the repository
    assert not any(f == os.path.basename(src) for _, _, fs in os.walk(ROOT) for f in fs)


def _write_pcd(path, pts, nrm, binary):
    n = pts.shape[0]
    hdr = ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\n"
           "FIELDS x y z rgb normal_x normal_y normal_z curvature\nSIZE 4 4 4 4 4 4 4 4\nTYPE F F F U F F F F\n"
           f"COUNT 1 1 1 1 1 1 1 1\nWIDTH {n}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {n}\n")
    rec = np.zeros(n, dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("rgb", "<u4"), ("nx", "<f4"), ("ny", "<f4"),
                             ("nz", "<f4"), ("c", "<f4")])
    rec["x"], rec["y"], rec["z"] = pts[:, 0], pts[:, 1], pts[:, 2]
    rec["nx"], rec["ny"], rec["nz"] = nrm[:, 0], nrm[:, 1], nrm[:, 2]
    rec["rgb"] = 0x00804020
    with open(path, "wb") as f:
        if binary:
            f.write((hdr + "DATA binary\n").encode())
            f.write(rec.tobytes())
        else:
            f.write((hdr + "DATA ascii\n").encode())
            for r in rec:
                f.write(("%.9g %.9g %.9g %d %.9g %.9g %.9g %.9g\n" % tuple(r)).encode())


def _voxel_grid(pts, nrm, leaf):
    """pcl::VoxelGrid (compat pcl/filters/voxel_grid.h) restated in numpy: per non-empty leaf,
    in increasing leaf index, the float mean (cloud-order sums) of x, y, z and the normal."""
    inv = np.float32(1.0) / np.float32(leaf)
    mnb = np.floor(pts.min(0) * inv).astype(np.int64)
    mxb = np.floor(pts.max(0) * inv).astype(np.int64)
    div = mxb - mnb + 1
    ijk = np.floor(pts * inv).astype(np.int64) - mnb
    idx = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
    order = np.argsort(idx, kind="stable")
    P, N = [], []
    s = 0
    while s < len(order):
        e = s
        while e < len(order) and idx[order[e]] == idx[order[s]]:
            e += 1
        acc = np.zeros(6, np.float32)
        for i in order[s:e]:
            acc[:3] += pts[i]
            acc[3:] += nrm[i]
        P.append(acc[:3] / np.float32(e - s))
        N.append(acc[3:] / np.float32(e - s))
        s = e
    return np.array(P, np.float32), np.array(N, np.float32)


def _voxel_grid_first(pts, nrm, leaf):
    P, N = _voxel_grid(pts, nrm, leaf)
    return P[0], N[0]


def _oracle_volume(oracle, pts, nrm, per_m):
    lo, hi = pts.min(0), pts.max(0)
    ov = oracle.Volume()
    ov.setDimensions(float(lo[0]), float(hi[0]), float(lo[1]), float(hi[1]), float(lo[2]), float(hi[2]))
    ov.setVolumeSize(*[int(np.float32(hi[i] - lo[i]) * np.float32(per_m)) for i in range(3)])
    ov.constructVolume()
    ov.integratePointCloud(pts, nrm)
    return ov


def _parse_dump(path):
    d = {"voxels": [], "cameras": []}
    for line in open(path):
        f = line.split()
        if f[0] == "bounds":
            d["bounds"] = [float(x) for x in f[1:7]]
        elif f[0] == "dims":
            d["dims"] = tuple(int(x) for x in f[1:4])
        elif f[0] == "camera":
            d["cameras"].append(np.array([float(x) for x in f[2:14]], np.float32))
        elif f[0] == "voxel":
            d["voxels"].append((int(f[1]), int(f[2]), int(f[3])))
    return d


@pytest.mark.gpu
@pytest.mark.parametrize("binary", [False, True])
def test_reference_raytracing_cpp_runs_headless(tmp_path, oracle, binary):
    assert os.path.exists(BINARY), "build it: python -c 'import __graft_entry__ as g; g.build()'"
    pts, nrm = Hh.cloud()
    pts, nrm = pts[::3].copy(), nrm[::3].copy()
    pcd = tmp_path / "cloud.pcd"
    _write_pcd(pcd, pts, nrm, binary)
    dump = tmp_path / "viz.txt"
    r = subprocess.run([BINARY, str(pcd)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, DMF_COMPAT_VIZ_DUMP=str(dump)))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Volume Integrated" in r.stdout and "Pointcloud Parsed" in r.stdout
    d = _parse_dump(dump)
    # Raytracing.cpp:62-75 on the oracle
    lo, hi = pts.min(0), pts.max(0)
    assert np.allclose(d["bounds"], [lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]], rtol=0, atol=0)
    ov = oracle.Volume()
    ov.setDimensions(float(lo[0]), float(hi[0]), float(lo[1]), float(hi[1]), float(lo[2]), float(hi[2]))
    ov.setVolumeSize(*[int(np.float32(hi[i] - lo[i]) * np.float32(125)) for i in range(3)])
    ov.constructVolume()
    ov.integratePointCloud(pts, nrm)
    assert d["dims"] == tuple(ov.dims)
    occ = ov.occupied_cells_
    assert [v[0] for v in d["voxels"]] == [int(h) for h in occ] and len(occ) > 1000
    # Raytracing.cpp:79-81: camera 0 = positionCameras(downsample(cloud, 0.3))[0]
    p0, n0 = _voxel_grid_first(pts, nrm, 0.3)
    T0 = scene.reference_style_poses(p0[None], n0[None], 300)[0]
    assert len(d["cameras"]) == 1 and np.array_equal(d["cameras"][0], T0)
    # Raytracing.cpp:90: reverseRayTraceFast(volume, camera 0, viz = true)
    eng = oracle.Engine(K_REF.ravel())
    found, good = eng.reverseRayTraceFast(ov, T0, True)
    view, goodf, _, _ = ov.voxel_table()
    got_view = np.array([v[1] for v in d["voxels"]])
    got_good = np.array([v[2] for v in d["voxels"]])
    assert np.array_equal(got_view, view[:len(occ)]) and np.array_equal(got_good, goodf[:len(occ)].astype(int))
    assert got_view.sum() > 0


def _read_pose_file(path):
    lines = open(path).read().split()
    n = int(lines[0])
    rows = [np.array([float(x) for x in ln.split(",")], np.float32) for ln in lines[1:1 + 3 * n]]
    return np.array(rows, np.float32).reshape(n, 12)


@pytest.mark.gpu
def test_reference_setcover_cpp_runs_headless(tmp_path, oracle):
    assert os.path.exists(BINARY_SC), "build it: python -c 'import __graft_entry__ as g; g.build()'"
    pts, nrm = Hh.cloud()
    pts, nrm = pts[::2].copy(), nrm[::2].copy()
    pcd = tmp_path / "cloud.pcd"
    _write_pcd(pcd, pts, nrm, True)
    out = tmp_path / "selected.txt"
    r = subprocess.run([BINARY_SC, str(pcd), str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    got = _read_pose_file(out)
    # SetCover.cpp:256-312 on the oracle
    ov = _oracle_volume(oracle, pts, nrm, 63)
    P, N = _voxel_grid(pts, nrm, 0.1)
    cams = scene.reference_style_poses(P, N, 500)
    cams = cams[cams.reshape(-1, 3, 4)[:, 2, 3] >= 0]  # filterCameras
    eng = oracle.Engine(K_REF.ravel())
    sets = [np.sort(eng.reverseRayTraceFast(ov, T, False)[1]) for T in cams]
    sel = [int(x) for x in oracle.greedy_set_cover(sets, 5)]
    assert len(sel) > 0 and len(cams) > len(sel)
    assert "Cameras found: %d" % len(sel) in r.stdout
    # writeCameraLocations (FileRoutines.hpp:98-112) streams with ostream's default %g (6 digits)
    exp = np.array([[np.float32(float("%g" % v)) for v in row] for row in cams[sel]], np.float32)
    assert np.array_equal(got, exp)
