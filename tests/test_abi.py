"""The C ABI library builds for gfx950, loads, and exports exactly what
include/hgx.h declares. No compute is called (no GPU here)."""

import ctypes
import os
import shutil

import pytest

from hypergraphembedding_amd import _hgx, build


@pytest.fixture(scope="module")
def lib_path():
  if not os.path.exists(build.LIB) and shutil.which("hipcc") is None \
      and not os.path.exists("/opt/rocm/bin/hipcc"):
    pytest.skip("no hipcc and no prebuilt libhgx.so")
  return build.build()


def test_every_declared_symbol_is_exported_and_bound(lib_path):
  declared = set(_hgx.header_symbols())
  assert len(declared) >= 25
  lib = ctypes.CDLL(lib_path)
  for name in declared:
    assert hasattr(lib, name), f"{name} declared in include/hgx.h but not exported"
  # the ctypes binding covers the header one to one
  assert declared == set(_hgx.SIGNATURES), declared ^ set(_hgx.SIGNATURES)
  _hgx.lib()  # binds every signature


def test_version_and_error_codes(lib_path):
  lib = _hgx.lib()
  assert lib.hgx_version() >= 1
  assert lib.hgx_last_error(None) == b"null context"


def test_no_silent_cpu_fallback(lib_path):
  """Without a usable HIP device the context refuses to exist."""
  import subprocess
  import sys
  code = ("import sys; sys.path.insert(0, %r)\n"
          "from hypergraphembedding_amd import _hgx\n"
          "try:\n  _hgx.Context(0)\nexcept Exception as e:\n"
          "  print('RAISED', type(e).__name__)\nelse:\n  print('CREATED')\n"
          % os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
  env = dict(os.environ, HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="-1")
  out = subprocess.run([sys.executable, "-c", code], capture_output=True,
                       text=True, env=env, timeout=120).stdout
  assert "RAISED" in out, out


def test_build_outputs_gfx950_code_object(lib_path):
  import subprocess
  tool = "/opt/rocm/lib/llvm/bin/llvm-objdump"
  if not os.path.exists(tool):
    pytest.skip("no llvm-objdump")
  data = open(lib_path, "rb").read()
  assert b"gfx950" in data


def _header_error_codes():
  import re
  with open(_hgx.HEADER) as f:
    text = f.read()
  return {m.group(1): int(m.group(2))
          for m in re.finditer(r"#define (HGX_E[A-Z]+) (-\d+)", text)}


# the exception each HGX_E* code becomes (include/hgx.h:8-19)
EXPECTED_EXC = {"HGX_EINVAL": AssertionError, "HGX_EZERODIV": ZeroDivisionError,
                "HGX_EVALUE": ValueError, "HGX_ENUMERIC": FloatingPointError,
                "HGX_EHIP": RuntimeError, "HGX_ENOMEM": RuntimeError,
                "HGX_ESTATE": RuntimeError, "HGX_EUNSUP": RuntimeError}


def test_every_error_code_has_a_mapping():
  """Every HGX_E* the header defines maps to the documented exception in
  _hgx._raise, the module constants agree with the header, and the
  reference-side ctypes stub in INTEGRATION.md maps the same codes."""
  codes = _header_error_codes()
  assert set(codes) == set(EXPECTED_EXC), set(codes) ^ set(EXPECTED_EXC)
  for name, rc in codes.items():
    assert getattr(_hgx, name) == rc, name
    with pytest.raises(EXPECTED_EXC[name]) as ei:
      _hgx._raise(rc, "x")
    if EXPECTED_EXC[name] is RuntimeError:  # not a narrower mapping
      assert type(ei.value) is _hgx.HgxError
  doc = open(os.path.join(os.path.dirname(_hgx.HEADER), "..",
                          "INTEGRATION.md")).read()
  for name, exc in EXPECTED_EXC.items():
    if exc is not RuntimeError:
      assert f"{codes[name]}: {exc.__name__}" in doc, name
