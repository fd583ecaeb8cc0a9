"""INTEGRATION.md's maintainer-facing binding stays in step with include/nngp.h (host test, no GPU).

The ctypes stub a pyNNGP maintainer would paste declares argtypes for the
C entry points and asserts the ABI revision; a stale snippet fails on import in the reference (the
round-5 snippet asserted revision 2 against a revision-3 header).  Here every `argtypes` list in the
document's python blocks is compared with the prototype in include/nngp.h, the asserted revision
with NNGP_ABI_VERSION and the built library's nngp_abi_version(), PLAN_INFO_LEN with
NNGP_PLAN_INFO_LEN, and pynngp_amd._lib's own argtypes with the header as well.
"""
import ctypes
import os
import re

import pytest

ROOT = os.path.join(os.path.dirname(__file__), "..")
HEADER = os.path.join(ROOT, "include", "nngp.h")
DOC = os.path.join(ROOT, "INTEGRATION.md")

# C parameter type -> the code the bindings use (P, I32, I64, D, SZ, U32, U64)
# (size_t and uint64_t are one ctypes type on LP64 Linux: both "SZ")
_SCALARS = {"int32_t": "I32", "int64_t": "I64", "double": "D", "size_t": "SZ", "uint32_t": "U32", "uint64_t": "SZ",
            "int": "I32", "float": "F"}


def _header_prototypes():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    src = re.sub(r"//[^\n]*", " ", src)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w \t\*]*?)\b(nngp_\w+)\s*\(([^;{]*?)\)\s*;", src, flags=re.S):
        name, args = m.group(2), " ".join(m.group(3).split())
        if args in ("", "void"):
            protos[name] = []
            continue
        codes = []
        for a in args.split(","):
            a = a.strip()
            if "*" in a:
                codes.append("P")
                continue
            toks = [t for t in a.replace("const", " ").split() if t]
            assert toks and toks[0] in _SCALARS, (name, a)
            codes.append(_SCALARS[toks[0]])
        protos[name] = codes
    return protos


def _header_define(name):
    m = re.search(rf"#define\s+{name}\s+(\d+)", open(HEADER).read())
    assert m, name
    return int(m.group(1))


def _doc_python():
    return "\n".join(re.findall(r"```python\n(.*?)```", open(DOC).read(), flags=re.S))


def test_header_parses():
    protos = _header_prototypes()
    assert len(protos) > 40
    assert protos["nngp_bf_sweep"][:3] == ["P", "I64", "I32"] and protos["nngp_abi_version"] == []


def test_doc_argtypes_match_header():
    protos = _header_prototypes()
    code = _doc_python()
    found = re.findall(r"_lib\.(nngp_\w+)\.argtypes\s*=\s*\[([^\]]*)\]", code)
    assert len(found) >= 8, found
    for name, lst in found:
        assert name in protos, f"INTEGRATION.md binds {name}, which include/nngp.h does not declare"
        doc = [t.strip() for t in lst.split(",") if t.strip()]
        assert doc == protos[name], f"{name}: INTEGRATION.md argtypes {doc} != include/nngp.h {protos[name]}"


def test_doc_abi_and_plan_info_match_header():
    code = _doc_python()
    m = re.search(r"assert _lib\.nngp_abi_version\(\) == (\d+)", code)
    assert m, "INTEGRATION.md's binding must assert the ABI revision"
    assert int(m.group(1)) == _header_define("NNGP_ABI_VERSION")
    m = re.search(r"PLAN_INFO_LEN = (\d+)", code)
    assert m and int(m.group(1)) == _header_define("NNGP_PLAN_INFO_LEN")


def test_library_abi_matches_header():
    from pynngp_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    lib = _lib.load()
    assert lib.nngp_abi_version() == _header_define("NNGP_ABI_VERSION")
    assert _lib.ABI_VERSION == _header_define("NNGP_ABI_VERSION")
    assert _lib.PLAN_INFO_LEN == _header_define("NNGP_PLAN_INFO_LEN")


_CT = {ctypes.c_void_p: "P", ctypes.c_int32: "I32", ctypes.c_int64: "I64", ctypes.c_double: "D",
       ctypes.c_size_t: "SZ", ctypes.c_uint32: "U32", ctypes.c_float: "F"}


def test_lib_binding_argtypes_match_header():
    """pynngp_amd._lib's own ctypes declarations (the binding the package itself uses)"""
    from pynngp_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    lib = _lib.load()
    protos = _header_prototypes()
    checked = 0
    for name, codes in protos.items():
        fn = getattr(lib, name, None)
        assert fn is not None, f"{name} declared in include/nngp.h but not exported"
        if fn.argtypes is None:
            continue
        got = [_CT.get(t, "P" if (t is not None and issubclass(t, (ctypes._Pointer, ctypes.c_char_p)))
                       else repr(t)) for t in fn.argtypes]
        assert got == codes, f"{name}: _lib argtypes {got} != include/nngp.h {codes}"
        checked += 1
    assert checked >= 30, checked
