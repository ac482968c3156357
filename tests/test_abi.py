"""CPU: the C-ABI library loads and exports every symbol include/dmf.h declares
(no compute: there is no GPU here), and fails loudly without a device."""
import ctypes as C

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
