"""C-ABI library: loads here (no GPU) and exports every symbol include/orbslam2_amd.h declares;
the product path fails loudly without it.  CPU only — no compute calls."""
import ctypes
import os
import re
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "orbslam2_amd.h"
LIB = ROOT / "orb_slam2_refactored_amd" / "liborbslam2_amd.so"


def declared_symbols():
    text = re.sub(r"/\*.*?\*/", " ", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(orb\w+)\s*\(", text, flags=re.M)))


@pytest.mark.skipif(not LIB.exists(), reason="library not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(str(LIB))
    syms = declared_symbols()
    assert len(syms) >= 18
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from orb_slam2_refactored_amd import _lib
    assert set(declared_symbols()) <= set(_lib.SIGNATURES)


def test_product_fails_loudly_without_library(tmp_path):
    code = ("import orb_slam2_refactored_amd as m\n"
            "try:\n    m.ORBextractor()\nexcept Exception as e:\n    print('RAISED', type(e).__name__)\n")
    env = dict(os.environ, ORBSLAM2_AMD_LIB=str(tmp_path / "missing.so"), PYTHONPATH=str(ROOT))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert "RAISED OrbError" in out.stdout, out.stdout + out.stderr


def test_package_does_not_import_oracle():
    """The product (the package, its native sources and bench.py's timed path) never imports, loads or
    executes the oracle: no `import oracle_api` / `from oracle...`, no ctypes / CDLL load of
    liborb_oracle, no subprocess into oracle/.  bench.py may use it only in its cpu_baseline legs."""
    bad = [re.compile(r"^\s*(import|from)\s+(oracle_api|oracle)\b", re.M),
           re.compile(r"liborb_oracle"),
           re.compile(r"oracle/_build"),
           re.compile(r"CDLL\([^)]*oracle", re.I),
           re.compile(r"subprocess\.[a-z_]+\([^)]*oracle", re.I)]
    for p in (ROOT / "orb_slam2_refactored_amd").rglob("*.py"):
        src = p.read_text()
        for rx in bad:
            assert not rx.search(src), (p, rx.pattern)
    for p in (ROOT / "orb_slam2_refactored_amd" / "csrc").glob("*"):
        if p.suffix in (".hip", ".h", ".cpp", ".inc"):
            src = p.read_text()
            assert "orb_oracle" not in src and "oracle_" not in src, p
    # bench.py: the oracle is reached only through oracle(), called only from cpu-baseline code
    src = (ROOT / "bench.py").read_text()
    assert "liborb_oracle" not in src
    body = src[src.index("def main():"):]
    assert "oracle" not in body.replace("cpu_baseline", "").replace("oracle/orb_oracle.cpp", ""), \
        "main() must not touch the oracle outside the cpu-baseline helpers"
    for m in re.finditer(r"(?<!def )oracle\(\)", src):
        fn = src[:m.start()].rsplit("\ndef ", 1)[-1].split("(", 1)[0]
        assert fn.startswith("cpu_") or fn.endswith("_leg") or fn == "oracle", fn


def test_cpp_wrapper_compiles_and_links(tmp_path):
    """include/orbslam2_amd.hpp (the C++ drop-in classes) compiles and links against the library."""
    src = ROOT / "tests" / "native" / "cpp_wrapper_use.cpp"
    obj = tmp_path / "w.o"
    subprocess.run(["g++", "-std=c++14", "-c", f"-I{ROOT / 'include'}", str(src), "-o", str(obj)], check=True)
    if LIB.exists():
        main = tmp_path / "main.cpp"
        main.write_text("int use_wrapper(); int main() { return use_wrapper() >= 0 ? 0 : 1; }\n")
        exe = tmp_path / "w"
        subprocess.run(["g++", str(main), str(obj), "-o", str(exe), f"-L{LIB.parent}", "-lorbslam2_amd",
                        f"-Wl,-rpath,{LIB.parent}"], check=True)
