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
    subprocess.run([gxx, "-std=c++17", "-fsyntax-only", "-Wall", "-I", compat, "-I", os.path.join(root, "include"),
                    str(src)], check=True, capture_output=True, text=True)
