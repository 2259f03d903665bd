"""The C-ABI boundary (include/octsam.h): liboctsam_hip.so loads without a GPU, exports every entry point
the header declares, and the Python binding table (_lib._SIGNATURES) covers exactly that set. No compute
calls here (no GPU in the build container)."""
import os
import re

import pytest

from dilabhelmholtzoct_amd import _lib

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "octsam.h")


def declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return sorted(set(re.findall(r"\b(octsam_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared()
    assert "octsam_gemm" in names and "octsam_cubical_ph" in names and "octsam_adam" in names
    assert len(names) >= 30


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_table_matches_header():
    assert sorted(_lib._SIGNATURES) == declared()


def test_abi_version_and_error_channel():
    lib = _lib.load()
    import re
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                            "octsam.h")).read()
    assert lib.octsam_abi_version() == int(re.search(r"#define OCTSAM_ABI_VERSION (\d+)", hdr).group(1)) == 20
    assert isinstance(lib.octsam_last_error(), (bytes, type(None)))


def test_gemm_rejects_bad_arguments_without_launching():
    """Argument validation happens on the host before any launch: a K-contiguous operand with K % 8 != 0
    must fail with a message, not fault."""
    lib = _lib.load()
    a = _lib.GemmArgs()
    a.M, a.N, a.K, a.batch = 64, 64, 6, 1
    a.lda, a.ldb, a.ldc = 6, 6, 64
    a.alpha = 1.0
    rc = lib.octsam_gemm(a, None)
    assert rc != 0
    assert lib.octsam_last_error()
