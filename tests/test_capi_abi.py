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
