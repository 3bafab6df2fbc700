"""The C-ABI library loads without a GPU and exports every symbol include/avr.h declares."""
import ctypes
import os
import re
import subprocess

from acceleratedvolrenderer_amd import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "avr.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(avr_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for must in ("avr_context_create", "avr_medium_grid", "avr_lights", "avr_camera", "avr_film", "avr_render",
                 "avr_film_read", "avr_last_error"):
        assert must in syms


def test_library_exports_every_declared_symbol():
    lib = capi.load()
    out = subprocess.check_output(["nm", "-D", "--defined-only", capi.LIB_PATH]).decode()
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    for sym in declared_symbols():
        assert sym in exported, sym
        assert getattr(lib, sym) is not None


def test_binding_covers_every_symbol():
    assert sorted(capi.SIGNATURES) == declared_symbols()


def test_errors_are_reported_not_raised():
    lib = capi.load()
    # no device context needed: argument validation fails first
    assert lib.avr_context_create(0, 0, None) != 0
    assert b"null" in lib.avr_last_error()
    assert lib.avr_render(None, 0, 1, 0, 5) != 0


def test_film_reduce_argument_errors_without_a_gpu():
    lib = capi.load()
    assert lib.avr_film_reduce_rccl(None, 1, 0) != 0
    assert b"context list" in lib.avr_last_error()


def _prototypes():
    """name -> (return type, [parameter types]) parsed from include/avr.h."""
    text = open(os.path.join(ROOT, "include", "avr.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"#[^\n]*", "", text)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(avr_[a-z_0-9]+)\s*\(([^;{]*?)\)\s*;", text):
        ret, name, params = m.group(1).strip(), m.group(2), m.group(3).strip()
        plist = [] if params in ("", "void") else [p.strip() for p in params.split(",")]
        protos[name] = (ret, plist)
    return protos


def _c_kind(decl):
    """Canonical kind of a C parameter declaration: scalar type, or ptr:<pointee>."""
    decl = re.sub(r"\bconst\b", " ", decl)
    array = "[" in decl
    decl = re.sub(r"\[[^\]]*\]", "", decl)
    stars = decl.count("*") + (1 if array else 0)
    words = decl.replace("*", " ").split()
    base = " ".join(words[:-1]) if len(words) > 1 and (stars or len(words) > 1) else " ".join(words)
    if not stars and len(words) == 1:      # a return type
        base = words[0]
    scalars = {"int": "i32", "long long": "i64", "float": "f32", "double": "f64", "void": "void",
               "char": "i8", "unsigned long long": "u64"}
    b = scalars.get(base, "struct:" + base)
    if stars == 0:
        return b
    return "ptr" * stars + ":" + b


def _ct_kind(t):
    """Canonical kind of a ctypes type (None = void)."""
    if t is None:
        return "void"
    simple = {ctypes.c_int: "i32", ctypes.c_longlong: "i64", ctypes.c_float: "f32", ctypes.c_double: "f64",
              ctypes.c_void_p: "ptr:void", ctypes.c_char_p: "ptr:i8", ctypes.c_ulonglong: "u64"}
    if t in simple:
        return simple[t]
    if hasattr(t, "_type_") and isinstance(t._type_, type):
        inner = _ct_kind(t._type_)
        if inner.startswith("ptr"):
            return "ptr" + inner
        return "ptr:" + inner
    if isinstance(t, type) and issubclass(t, ctypes.Structure):
        return "struct:" + t.__name__
    raise AssertionError(f"unmapped ctypes type {t}")


_STRUCTS = {"AvrStats": "avr_stats", "AvrVdbGrid": "avr_vdb_grid", "AvrGraphSampling": "avr_graph_sampling"}


def _compatible(c, py):
    """A ctypes argtype matches its C parameter when the kinds are equal; opaque handles
    (avr_context *, avr_graph *) and device pointers bind as c_void_p."""
    for k, v in _STRUCTS.items():
        py = py.replace("struct:" + k, "struct:" + v)
    if c == py:
        return True
    if py == "ptr:void" and c.startswith("ptr:") and not c.startswith("ptrptr"):
        return True        # any single-level data pointer / handle passed as an address
    if py == "ptrptr:void" and c.startswith("ptrptr:"):
        return True        # handle out-parameters (avr_context **, void **)
    return False


def test_binding_prototypes_match_the_header():
    """capi.SIGNATURES agrees with every prototype in include/avr.h in arity and in each
    parameter's scalar type / pointee (ctypes alone cannot detect that drift)."""
    protos = _prototypes()
    assert sorted(protos) == declared_symbols()
    bad = []
    for name, (ret, params) in protos.items():
        res, args = capi.SIGNATURES[name]
        if len(params) != len(args):
            bad.append(f"{name}: {len(params)} parameters in avr.h, {len(args)} in capi.SIGNATURES")
            continue
        if not _compatible(_c_kind(ret), _ct_kind(res)):
            bad.append(f"{name}: returns {ret} vs {res}")
        for i, (p, a) in enumerate(zip(params, args)):
            if not _compatible(_c_kind(p), _ct_kind(a)):
                bad.append(f"{name} arg {i}: {p!r} ({_c_kind(p)}) vs {a} ({_ct_kind(a)})")
    assert not bad, "\n".join(bad)


def test_header_compiles_as_c_and_cpp(tmp_path):
    """include/avr.h is a plain C header: a C caller (tests/capi_smoke.c) compiles with gcc
    and links against libavr_hip.so without a GPU (it runs in tests/test_gpu_capi_caller.py)."""
    capi.load()
    exe = tmp_path / "capi_smoke"
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "capi_smoke.c"), "-o", str(exe),
                           "-L", os.path.dirname(capi.LIB_PATH), "-lavr_hip",
                           "-Wl,-rpath," + os.path.dirname(capi.LIB_PATH), "-lm"])
    src = tmp_path / "hdr.cpp"
    src.write_text('#include "avr.h"\nint main() { return avr_last_error() == nullptr; }\n')
    subprocess.check_call(["g++", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           "-c", str(src), "-o", str(tmp_path / "hdr.o")])
