"""CPU checks of the C-ABI library: it loads and exports every declared symbol."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dls_hip.h")
LIB = os.path.join(ROOT, "distributed_learning_simulator_amd", "libdls_hip.so")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dls_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail("libdls_hip.so is not built (run __graft_entry__.build())")
    return ctypes.CDLL(LIB)


def test_header_declares_entry_points():
    names = declared_functions()
    assert "dls_fedavg_f32" in names and "dls_sign_vote" in names and len(names) >= 15


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_matches_header():
    from distributed_learning_simulator_amd import _native
    assert set(_native.SIGNATURES) == set(declared_functions())


def test_abi_version_and_error_without_gpu(lib):
    lib.dls_abi_version.restype = ctypes.c_int
    assert lib.dls_abi_version() == 2
    lib.dls_last_error.restype = ctypes.c_char_p
    # argument validation happens before any device call
    lib.dls_fedavg_f32.restype = ctypes.c_int
    rc = lib.dls_fedavg_f32(None, ctypes.c_int64(0), None, None, 0, ctypes.c_float(1.0),
                            ctypes.c_int64(0), 0, None, None)
    assert rc == -1
    assert b"null pointer" in lib.dls_last_error()


def test_dequant_rejects_bad_mode_without_gpu(lib):
    """dls_dequant_fedavg_mode validates its mode (DLS_FEDAVG_EXACT / _FMA) and the
    tile-group counts before any device call (no pointer is dereferenced on the
    host)."""
    f = lib.dls_dequant_fedavg_mode
    f.restype = ctypes.c_int
    dummy = ctypes.c_void_p(16)  # never dereferenced: validation comes first
    nfast = (ctypes.c_int32 * 10)(*[0] * 7, 1, 0, 0)
    for mode, what in ((2, b"mode"), (-1, b"mode")):
        rc = f(dummy, 1, nfast, dummy, ctypes.c_int64(1024), None, ctypes.c_int64(4), dummy,
               ctypes.c_int64(1), ctypes.c_int64(1), dummy, dummy, 1, ctypes.c_float(1.0),
               mode, dummy, None)
        assert rc == -1 and what in lib.dls_last_error()
    bad = (ctypes.c_int32 * 10)(*[0] * 7, -1, 0, 0)
    rc = f(dummy, 1, bad, dummy, ctypes.c_int64(1024), None, ctypes.c_int64(4), dummy,
           ctypes.c_int64(1), ctypes.c_int64(1), dummy, dummy, 1, ctypes.c_float(1.0), 0, dummy,
           None)
    assert rc == -1 and b"nfast[7]" in lib.dls_last_error()


def test_conv_rejects_bad_shapes_without_gpu():
    """The convolution entry points validate shapes and alignment before any
    device call (the pointers below are never dereferenced)."""
    from distributed_learning_simulator_amd import _native
    L = _native.lib()
    d = ctypes.c_void_p(256)  # 16-byte aligned, never dereferenced
    # C = 48: not a multiple of 32
    rc = L.dls_conv_bn_act_split(d, 2, 8, 8, 48, d, 64, 3, 3, 1, 1, None, None, 1, d, None)
    assert rc == -1 and b"multiple of 32" in L.dls_last_error()
    # Cout = 96: not a multiple of 64
    rc = L.dls_conv_bn_act_split(d, 2, 8, 8, 64, d, 96, 3, 3, 1, 1, None, None, 1, d, None)
    assert rc == -1 and b"Cout" in L.dls_last_error()
    # misaligned output
    rc = L.dls_conv_bn_act_split(d, 2, 8, 8, 64, d, 64, 3, 3, 1, 1, None, None, 1,
                                 ctypes.c_void_p(258), None)
    assert rc == -2 and b"alignment" in L.dls_last_error()
    # a stem whose reduction exceeds one 32-deep chunk (4 channels x 3 x 3 = 36)
    rc = L.dls_conv_stem_bn_act_f32(d, 2, 4, 8, 8, d, 64, 3, 3, 1, 1, None, 1, d, None)
    assert rc == -1 and b"KH*KW*C" in L.dls_last_error()
    rc = L.dls_conv_pack_im2col_f32(d, 2, 3, 8, 8, 3, 3, 1, 1, 16, d, None)  # Kp < 27
    assert rc == -1
    rc = L.dls_pool_linear_split(d, 2, 16, 4096, d, None, 10, d, None)  # C > 2048
    assert rc == -1 and b"C <= 2048" in L.dls_last_error()
    assert _native.split_channels(3) == 32 and _native.split_channels(64) == 64


def test_split_conv_macs_counts_resnet18():
    """The MAC counts the bench's conv roofline uses: ResNet-18 at 32x32 has
    555,422,720 multiply-accumulates per image (the textbook 0.56 GMAC), and the
    library issues the stem's 27 -> 32 padding on top."""
    from distributed_learning_simulator_amd.models import ResNet18, split_conv_macs
    issued, useful = split_conv_macs(ResNet18(), 32, 32)
    assert useful == 555_422_720
    assert issued - useful == 32 * 32 * 64 * (32 - 27)


def test_inferencer_rejects_unknown_conv():
    import pytest
    import torch
    from distributed_learning_simulator_amd.models import LeNet5
    from distributed_learning_simulator_amd.trainer import Inferencer
    with pytest.raises(ValueError, match="conv"):
        Inferencer(LeNet5(), (torch.zeros(1, 1, 32, 32), torch.zeros(1, dtype=torch.long)),
                   device=torch.device("cpu"), conv="cudnn")


def test_product_path_has_no_oracle_import():
    """The shipped package must not import the CPU oracle (no CPU fallback)."""
    pkg = os.path.join(ROOT, "distributed_learning_simulator_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle\b", src, re.M), f


def test_two_constant_division_check_without_gpu(lib):
    """dls_two_constant_division's host-side exhaustive check agrees with an
    independent numpy restatement of fma(a, yh, RN(a*yl)) == RN(a/b) over every
    fp32 mantissa (float64 products are exact for the fma's 48-bit product)."""
    import numpy as np
    f = lib.dls_two_constant_division
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_float]
    a = (np.arange(1 << 23, dtype=np.uint32) | np.uint32(0x3F800000)).view(np.float32)
    for b in (55123.0, 49972.0, 1024.0, 3.0, 7.0, 100.0):
        b32 = np.float32(b)
        yh = np.float32(1.0 / float(b32))
        yl = np.float32(1.0 / float(b32) - float(yh))
        lo = (a * yl).astype(np.float32)  # RN(a*yl)
        # fma: exact a*yh + lo in float64 (a*yh has <= 48 significant bits; the
        # sum is exact unless exponents differ wildly, which they do not here),
        # then one rounding to fp32
        q = (a.astype(np.float64) * np.float64(yh) + np.float64(lo)).astype(np.float32)
        expect = int(np.array_equal(q, a / b32))
        assert f(b) == expect, b
    assert f(0.5) == 0  # outside the fast range: never two-constant


def test_library_built_from_this_tree(lib):
    """The loaded libdls_hip.so was compiled from exactly the sources in this tree
    (the source hash the Makefile compiles in)."""
    from distributed_learning_simulator_amd import _native
    lib.dls_source_hash.restype = ctypes.c_char_p
    assert lib.dls_source_hash().decode() == _native.source_hash()


def test_conv_wrappers_validate_operands_without_gpu():
    """conv_bn_act / conv_stem_bn_act / pool_linear reject operands the kernels
    would read or write out of bounds: the checks run before any
    pointer reaches the library, so CPU tensors exercise them here."""
    import torch
    from distributed_learning_simulator_amd import _native
    B, H, W, C, CO = 2, 4, 4, 64, 64
    x = torch.zeros(B, H, W, 2 * C, dtype=torch.int16)
    w = torch.zeros(CO, 2 * 9 * C, dtype=torch.int16)
    good = torch.zeros(4 * CO)
    for bad in (torch.zeros(3 * CO), torch.zeros(4 * CO, dtype=torch.float64),
                torch.zeros(8 * CO)[::2]):
        with pytest.raises(RuntimeError, match="consts"):
            _native.conv_bn_act(x, w, (3, 3), 1, 1, bad)
    res = torch.zeros(B, H, W, 2 * CO, dtype=torch.float16)
    with pytest.raises(RuntimeError, match="residual"):
        _native.conv_bn_act(x, w, (3, 3), 1, 1, good, res)
    with pytest.raises(RuntimeError, match="out must be"):
        _native.conv_bn_act(x, w, (3, 3), 1, 1, good, out=torch.zeros(B, H, W, CO, dtype=torch.int16))
    with pytest.raises(RuntimeError, match="alias x"):
        _native.conv_bn_act(x, w, (3, 3), 1, 1, good, out=x)
    r = torch.zeros(B, H, W, 2 * CO, dtype=torch.int16)
    with pytest.raises(RuntimeError, match="alias residual"):
        _native.conv_bn_act(x, w, (3, 3), 1, 1, good, r, out=r)
    xs = torch.zeros(B, 3, 8, 8)
    ws = torch.zeros(CO, 64, dtype=torch.int16)
    with pytest.raises(RuntimeError, match="consts"):
        _native.conv_stem_bn_act(xs, ws, (3, 3), 1, 1, torch.zeros(CO))
    with pytest.raises(RuntimeError, match="weight"):
        _native.pool_linear(x, torch.zeros(10, C, dtype=torch.bfloat16))
    with pytest.raises(RuntimeError, match="weight"):
        _native.pool_linear(x, torch.zeros(C, 10).t())
    with pytest.raises(RuntimeError, match="bias"):
        _native.pool_linear(x, torch.zeros(10, C), torch.zeros(10, dtype=torch.float16))
    with pytest.raises(RuntimeError, match="bias"):
        _native.pool_linear(x, torch.zeros(10, C), torch.zeros(20)[::2])


def test_library_sources_read_no_environment():
    """The kernels a coalition's utility runs through are chosen from the shapes
    alone: no product source reads the process environment (a probe knob is a
    compile-time macro, tools/build_variants.py), so two ranks cannot disagree on
    a utility because their environments differ."""
    csrc = os.path.join(ROOT, "distributed_learning_simulator_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".hip", ".h")):
            src = open(os.path.join(csrc, f)).read()
            assert "getenv" not in src, f
