"""The drop-in boundary without a GPU: libraries load, every declared entry
point is exported, the facade header keeps the reference's layouts, and the
library fails loudly (no CPU fallback) when no device is present."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import PKG, REPO

INC = os.path.join(REPO, "include")


def _declared(header):
    src = open(os.path.join(INC, header)).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(mas_\w+)\s*\(", src, re.M)))


def test_header_declarations_match_binding_list():
    import mas_amd
    assert _declared("mas_capi.h") == sorted(mas_amd.EXPORTS)


def test_library_exports_every_declared_symbol():
    import mas_amd
    lib = ctypes.CDLL(mas_amd.LIB_PATH)
    missing = [s for s in _declared("mas_capi.h") if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.mas_version() == 5


def test_facade_exports_reference_methods():
    import mas_amd
    out = subprocess.run(["nm", "-D", "-C", "--defined-only", mas_amd.FACADE_PATH], capture_output=True,
                         text=True, check=True).stdout
    for sym in ("SE::SeSchwarzPreconditioner::AllocatePrecoditioner(int, int, int)",
                "SE::SeSchwarzPreconditioner::Preconditioning(SE::SeVec3fSimd*, SE::SeVec3fSimd const*, int)",
                "SE::SeSchwarzPreconditioner::PreparePreconditioner(", "CPU_THREAD_NUM"):
        assert sym in out, sym


def test_facade_header_layouts_compile():
    src = os.path.join(REPO, "tests", "cpp", "layout_check.cpp")
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", INC, src], check=True)


def test_packed_inverse_slot_layout(tmp_path):
    """csrc/layout.h: slot_of inverts slot_ij over all 4656 slots (host g++ build)."""
    src = os.path.join(REPO, "tests", "cpp", "slot_layout_check.cpp")
    exe = str(tmp_path / "slotchk")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(PKG, "csrc"), src, "-o", exe], check=True)
    subprocess.run([exe], check=True)


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import mas_amd
    with pytest.raises(mas_amd.MasError, match="NO_DEVICE"):
        mas_amd.SeSchwarzPreconditioner()


def test_null_handle_and_bad_args():
    import mas_amd
    L = mas_amd.lib()
    assert L.mas_destroy(None) == -1
    assert L.mas_apply(None, None, None) == -1
    assert L.mas_create(None, None) == -1


def test_wrapper_operand_checks_without_gpu():
    """The binding refuses wrongly shaped / typed operands before any copy
    (the C ABI copies exactly nV*16, nnz*36, (nV+1)*4 bytes)."""
    import numpy as np
    import torch
    import mas_amd
    from mas_amd import _host, _dev, MasError
    ok = _host(np.zeros((5, 3, 3), np.float64), np.float32, 5, 9, "diag")
    assert ok.dtype == np.float32 and ok.flags.c_contiguous and ok.size == 45
    with pytest.raises(MasError, match="expected 5 x 4"):
        _host(np.zeros((5, 3), np.float32), np.float32, 5, 4, "r")
    with pytest.raises(MasError, match="torch tensor"):
        _host(torch.zeros(5, 4), np.float32, 5, 4, "r")
    assert _dev(1234, 5, 4, "float32", "z") == 1234  # raw pointers are the caller's contract
    with pytest.raises(MasError, match="not on a GPU"):
        _dev(torch.zeros(5, 4), 5, 4, "float32", "z")
    with pytest.raises(MasError, match="torch cuda tensor"):
        _dev(np.zeros((5, 4), np.float32), 5, 4, "float32", "z")
