"""CPU: the C-ABI library loads and exports every symbol include/dmf.h declares
(no compute: there is no GPU here), and fails loudly without a device."""
import ctypes as C
import os

import pytest


def test_header_symbols_exported():
    from dmf_amd import _lib
    L = _lib.load()
    syms = _lib.declared_symbols()
    assert len(syms) >= 40
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(_lib.SIGNATURES) == set(syms)


def test_abi_version_and_status_strings():
    from dmf_amd import _lib
    L = _lib.load()
    assert L.dmf_abi_version() == 1
    assert L.dmf_status_string(0) == b"ok"
    assert L.dmf_status_string(7) == b"no usable GPU"


def test_no_cpu_fallback_without_gpu():
    from dmf_amd import _lib
    import dmf_amd
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(dmf_amd.DmfError) as e:
        dmf_amd.VoxelVolume()
    assert e.value.status == _lib.DMF_ERR_NO_DEVICE


def test_null_arguments_rejected():
    from dmf_amd import _lib
    L = _lib.load()
    assert L.dmf_volume_get_info(None, None) == _lib.DMF_ERR_INVALID
    assert L.dmf_device_count(None) == _lib.DMF_ERR_INVALID
    assert L.dmf_volume_destroy(None) == 0


def test_compat_headers_compile(tmp_path):
    """The C++ drop-in headers (compat/) compile without Eigen/PCL, including the
    OccupancyGrid and Algorithms mirrors (g++ -fsyntax-only; no GPU needed)."""
    import shutil
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    compat = os.path.join(root, "depth-map-fusion-utils_amd", "compat")
    src = tmp_path / "use.cpp"
    src.write_text('''
#include "Algorithms.hpp"
#include "Camera.hpp"
#include "OccupancyGrid.hpp"
#include "RayTracingEngine.hpp"
#include "Volume.hpp"
int main() {
  OccupancyGrid g;
  g.setDimensions(-1, 1, -1, 1, -1, 1);
  g.setResolution(0.05f, 0.05f, 0.05f);
  g.setK(1);
  g.construct();
  auto c = std::make_shared<pcl::PointCloud<pcl::PointXYZRGB>>();
  auto n = std::make_shared<pcl::PointCloud<pcl::PointNormal>>();
  g.updateStates(c, n);
  auto out = std::make_shared<pcl::PointCloud<pcl::PointXYZRGBNormal>>();
  g.downloadHQCloud(out);
  g.downloadReorganizedCloud(out, true);
  VoxelVolume v;
  std::vector<std::vector<unsigned long long int>> sets;
  auto sel = Algorithms::greedySetCover(v, sets);
  sel = Algorithms::greedySetCover(sets);  // the reference signature (Algorithms.hpp:38)
  return (int)(out->points.size() + sel.size());
}
''')
    gxx = shutil.which("g++")
    assert gxx, "g++ is part of the image"
    subprocess.run([gxx, "-std=c++17", "-fsyntax-only", "-Wall", "-I", compat, "-I", os.path.join(compat, "shims"),
                    "-I", os.path.join(root, "include"), str(src)], check=True, capture_output=True, text=True)


def test_compat_real_library_configuration(tmp_path):
    """VERDICT r2 (boundary recipe): with DMF_COMPAT_REAL_EIGEN / DMF_COMPAT_REAL_PCL and
    compat/ FIRST on the include path, <Eigen/Dense> and the PCL headers
    resolve to the caller's libraries, not to anything inside compat/ (the headless shims
    live in compat/shims/, which that recipe leaves off the path).  Eigen and PCL are absent
    from this image, so stand-in "library" headers in a scratch include dir mark themselves
    and alias the lite types; the hot-path drop-ins must compile against them and see the
    markers."""
    import shutil
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    compat = os.path.join(root, "depth-map-fusion-utils_amd", "compat")
    for d in ("Eigen", "pcl", "boost"):
        assert not os.path.exists(os.path.join(compat, d)), f"compat/{d} would shadow the real library"
    lib = tmp_path / "libinc"
    (lib / "Eigen").mkdir(parents=True)
    (lib / "pcl").mkdir()
    (lib / "Eigen" / "Dense").write_text(
        "#pragma once\n#define SCRATCH_LIB_EIGEN 1\n"
        "namespace Eigen { using Affine3f = ::dmf_compat::Affine3f; using Vector3f = ::dmf_compat::Vector3f; }\n")
    (lib / "pcl" / "point_types.h").write_text(
        "#pragma once\n#define SCRATCH_LIB_PCL_TYPES 1\nnamespace pcl { using PointXYZ = ::dmf_compat::PointXYZ;\n"
        "using PointXYZRGB = ::dmf_compat::PointXYZRGB; using PointXYZRGBNormal = ::dmf_compat::PointXYZRGBNormal;\n"
        "using PointNormal = ::dmf_compat::PointNormal; using Normal = ::dmf_compat::Normal; }\n")
    (lib / "pcl" / "point_cloud.h").write_text(
        "#pragma once\n#define SCRATCH_LIB_PCL_CLOUD 1\n"
        "namespace pcl { template <class T> using PointCloud = ::dmf_compat::PointCloud<T>; }\n")
    src = tmp_path / "use_real.cpp"
    src.write_text('''
#include "Algorithms.hpp"
#include "Camera.hpp"
#include "OccupancyGrid.hpp"
#include "RayTracingEngine.hpp"
#include "Volume.hpp"
#include <Eigen/Dense>
#include <pcl/point_cloud.h>
#include <pcl/point_types.h>
#if !defined(SCRATCH_LIB_EIGEN) || !defined(SCRATCH_LIB_PCL_TYPES) || !defined(SCRATCH_LIB_PCL_CLOUD)
#error "a compat header shadowed the caller's Eigen / PCL"
#endif
int main() {
  VoxelVolume v;
  std::vector<float> K = {600, 0, 320, 0, 600, 240, 0, 0, 1};
  Camera cam(K);
  RayTracingEngine eng(cam);
  Eigen::Affine3f T = Eigen::Affine3f::Identity();
  auto r = eng.reverseRayTraceFast(v, T, false);
  RayTracingEngine::FusionCounts acc;
  std::vector<uint16_t> depth(640 * 480);
  eng.fuseDepth(v, depth, std::vector<Eigen::Affine3f>{T}, acc);
  return (int)r.second.size() + (int)eng.logOdds(v, acc).size();
}
''')
    gxx = shutil.which("g++")
    r = subprocess.run([gxx, "-std=c++17", "-fsyntax-only", "-Wall", "-DDMF_COMPAT_REAL_EIGEN", "-DDMF_COMPAT_REAL_PCL",
                        "-I", compat, "-I", str(lib), "-I", os.path.join(root, "include"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_pcd_reader_rejects_bad_headers(tmp_path):
    """the headless PCD reader (compat/shims/pcl/io/pcd_io.h) treats the file as
    untrusted: a field SIZE outside {1, 2, 4, 8} (TYPE U / I) or {4, 8} (TYPE F), or COUNT < 1,
    is rejected (-1) before any record is read; a well-formed binary file still loads.  Built
    with ASan + UBSan, so an overflow would fail the run."""
    import shutil
    import struct
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    shims = os.path.join(root, "depth-map-fusion-utils_amd", "compat", "shims")

    def pcd(fields, sizes, types, counts, payload):
        head = (f"VERSION .7\nFIELDS {fields}\nSIZE {sizes}\nTYPE {types}\nCOUNT {counts}\nWIDTH 1\nHEIGHT 1\n"
                f"POINTS 1\nDATA binary\n").encode()
        return head + payload
    good = pcd("x y z", "4 4 4", "F F F", "1 1 1", struct.pack("<fff", 1.0, 2.0, 3.0))
    cases = {"good.pcd": good,
             "u16.pcd": pcd("x y z", "4 4 16", "F F U", "1 1 1", b"\0" * 28),
             "i0.pcd": pcd("x y z", "4 4 0", "F F I", "1 1 1", b"\0" * 8),
             "f2.pcd": pcd("x y z", "4 4 2", "F F F", "1 1 1", b"\0" * 10),
             "count0.pcd": pcd("x y z", "4 4 4", "F F F", "1 1 0", b"\0" * 8),
             "typeq.pcd": pcd("x y z", "4 4 4", "F F Q", "1 1 1", b"\0" * 12)}
    for name, data in cases.items():
        (tmp_path / name).write_bytes(data)
    src = tmp_path / "pcd.cpp"
    src.write_text('''
#include <cstdio>
#include <pcl/io/pcd_io.h>
#include <pcl/point_types.h>
int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {
    pcl::PointCloud<pcl::PointXYZRGB> c;
    const int r = pcl::io::loadPCDFile(argv[i], c);
    std::printf("%d %zu %g\\n", r, c.points.size(), c.points.empty() ? 0.0 : (double)c.points[0].z);
  }
  return 0;
}
''')
    exe = tmp_path / "pcd"
    gxx = shutil.which("g++")
    subprocess.run([gxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I", shims, str(src), "-o", str(exe)], check=True, capture_output=True, text=True)
    names = list(cases)
    out = subprocess.run([str(exe)] + [str(tmp_path / n) for n in names], check=True, capture_output=True,
                         text=True).stdout.split("\n")
    res = dict(zip(names, out))
    assert res["good.pcd"] == "0 1 3"
    for n in names[1:]:
        assert res[n].startswith("-1 "), (n, res[n])
