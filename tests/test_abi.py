"""The C-ABI library loads and exports exactly what include/*.h declares; the
ctypes prototypes match the header; argument validation reports through
msp_last_error without touching a GPU."""
import ctypes
import glob
import os
import re

import pytest

from sparseconvnet import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declarations():
    decls = {}
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        for m in re.finditer(r"\b(msp_\w+)\s*\(([^)]*)\)\s*;", src):
            args = [a for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
            decls[m.group(1)] = len(args)
    return decls


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    decls = _declarations()
    assert len(decls) >= 30
    missing = [n for n in decls if not hasattr(lib, n)]
    assert not missing, missing


def _exported():
    """msp_* functions in the .so's dynamic symbol table (read from the ELF file; no tool needed)."""
    import struct
    data = open(_lib.LIB_PATH, "rb").read()
    assert data[:4] == b"\x7fELF" and data[4] == 2 and data[5] == 1  # 64-bit little-endian
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    out = set()
    for sec in secs:
        if sec[1] != 11:  # SHT_DYNSYM
            continue
        strtab = secs[sec[6]]
        for k in range(sec[5] // sec[9]):
            name_off, info, _, shndx, _, _ = struct.unpack_from("<IBBHQQ", data, sec[4] + k * sec[9])
            if shndx == 0 or (info & 0xF) != 2:  # defined functions only (STT_FUNC)
                continue
            s0 = strtab[4] + name_off
            name = data[s0:data.index(b"\0", s0)].decode()
            if name.startswith("msp_"):
                out.add(name)
    return out


def test_exports_are_exactly_the_header():
    """The product library exports no entry point the header does not declare (no experiment hooks, no
    process-global knobs: VERDICT r02 "stateless C-ABI"), and every declared one."""
    exported = _exported()
    decls = set(_declarations())
    assert exported == decls, (sorted(exported - decls), sorted(decls - exported))
    assert not any("debug" in n for n in exported)


def test_prototypes_match_header():
    decls = _declarations()
    assert set(decls) == set(_lib.PROTOTYPES)
    for name, n in decls.items():
        assert len(_lib.PROTOTYPES[name][1]) == n, name


def test_queries_and_validation_without_gpu():
    lib = _lib.load()
    assert lib.msp_abi_version() == 10
    assert _lib.query("msp_hash_capacity", 1000) == 2048
    assert _lib.query("msp_hash_capacity", 10) == 1024
    assert _lib.query("msp_scan_workspace_size", 5000) > 0
    assert _lib.query("msp_bn_partials", 10 ** 7, 32) == 1024
    assert _lib.query("msp_conv_tile_rows", 10 ** 6, 32, 32) == 128
    assert _lib.query("msp_conv_tile_rows", 10 ** 6, 64, 64) == 128
    # x6 form: split weights (K x 3 x c_out x c_pad bf16) + offset-split partials on small grids
    assert _lib.query("msp_conv_tile_workspace_size", 10 ** 6, 27, 64, 64, 128) == 27 * 3 * 64 * 64 * 2
    assert _lib.query("msp_conv_tile_workspace_size", 2000, 27, 192, 192, 128) > 27 * 3 * 192 * 192 * 2
    # narrow outputs: per-wave x6 form, weight images only (K x c_out x 32-deep k-slices x 3 pieces bf16)
    assert _lib.query("msp_conv_tile_workspace_size", 10 ** 6, 27, 32, 32, 128) == 27 * 32 * 32 * 6
    # invalid arguments are rejected before any HIP call
    rc = lib.msp_conv_tile(None, 3, None, 27, 0, 16, 64, None, None, None, None, 100, None, None, 0, None)
    assert rc == -1 and b"multiples of 16" in lib.msp_last_error()
    rc = lib.msp_conv_tile(None, 16, None, 27, 0, 16, 96, None, None, None, None, 100, None, None, 0, None)
    assert rc == -1 and b"tile_rows" in lib.msp_last_error()
    rc = lib.msp_conv_tile(None, 16, None, 27, 0, 16, 64, None, None, None, None, 100, None, None, 0, None)
    assert rc == -1 and b"must be 128" in lib.msp_last_error()
    rc = lib.msp_conv_tile(None, 3, None, 27, 0, 16, 64, None, None, None, None, 100, None, None, 0, None)
    assert rc == -1 and b"multiples of 16" in lib.msp_last_error()
    rc = lib.msp_subm_map(None, 10, 12, 4096, 4, None, 1024, None, None)
    assert rc == -1 and b"odd" in lib.msp_last_error()
    rc = lib.msp_down_map(None, 10, None, 12, 3, None, 5, None)
    assert rc == -1
    with pytest.raises(RuntimeError, match="msp_tile_rulebook"):
        _lib.call("msp_tile_rulebook", None, 300, 10, 64, None, None, None, None, 0, None, 0, None)
    with pytest.raises(RuntimeError, match="tile_rows"):
        _lib.call("msp_tile_rulebook", None, 27, 10, 32, None, None, None, None, 0, None, 0, None)
