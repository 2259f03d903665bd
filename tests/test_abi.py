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
    assert lib.octsam_abi_version() == int(re.search(r"#define OCTSAM_ABI_VERSION (\d+)", hdr).group(1)) == 24
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


def test_round4_entries_reject_bad_arguments_without_launching():
    """The round-4 entry points validate on the host before any launch (no GPU needed): null operands, a chunk
    length that does not divide L, a row stride below the row width each fail with a message."""
    lib = _lib.load()
    fake = 1 << 20  # a non-null, 16-B aligned address that is never dereferenced (validation fails first)
    # t2i / i2t backwards with the prompt sum fused in: L % 64 != 0
    rc = lib.octsam_dec_t2i_bwd_sum(fake, fake, fake, 384, 3, 6, 7, 4000, fake, fake, fake, fake, fake, fake, 256,
                                    fake, None)
    assert rc != 0 and b"t2i_bwd_sum" in lib.octsam_last_error()
    rc = lib.octsam_dec_i2t_bwd_sum(fake, 384, 3, fake, fake, 6, 7, 4000, fake, 128, fake, 128, fake, None)
    assert rc != 0 and b"i2t_bwd_sum" in lib.octsam_last_error()
    # the strided mask-head backward: a row stride below 256
    rc = lib.octsam_upmask_ln_bwd_strided(fake, fake, fake, fake, fake, 4, 1, fake, fake, fake, fake, fake, fake, 128,
                                          fake, fake, fake, fake, fake, fake, None)
    assert rc != 0 and b"strided" in lib.octsam_last_error()
    # null operand
    rc = lib.octsam_dec_t2i_bwd_sum(None, fake, fake, 384, 3, 6, 7, 4096, fake, fake, fake, fake, fake, fake, 256,
                                    fake, None)
    assert rc != 0
    # sizes of the workspaces / partials the entries expect
    assert lib.octsam_dec_t2i_bwd_sum_workspace(168, 7, 4096) == 168 * 64 * 4 * 256 + 168 * 8 * 7 * 2
    assert lib.octsam_dec_i2t_bwd_sum_partials(168, 7, 4096) == 64 * 168 * 2 * 7 * 128
