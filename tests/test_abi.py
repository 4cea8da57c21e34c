"""C-ABI checks that need no GPU: the library loads and exports every entry
point ``include/transmil_hip.h`` declares; the ctypes table matches; no compute."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "transmil_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(tm_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "tm_gemm" in syms and "tm_pinv_fwd" in syms and "tm_nys_a1_bwd" in syms
    assert len(syms) >= 35


def test_library_exports_every_declared_symbol():
    from transmil_deepgraft_amd import _lib
    lib = _lib.lib()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_ctypes_table_covers_header():
    from transmil_deepgraft_amd import _lib
    assert set(declared_symbols()) == set(_lib.EXPORTED)


def test_struct_layouts_match_c(tmp_path):
    """Every field offset of the ctypes mirrors equals the C compiler's offsetof()."""
    import shutil
    import subprocess
    from transmil_deepgraft_amd._lib import GemmArgs, BmmJob, OptimTensor, OptimTable, CastTable
    structs = (("tm_gemm_args", GemmArgs), ("tm_bmm_job", BmmJob), ("tm_optim_tensor", OptimTensor),
               ("tm_optim_table", OptimTable), ("tm_cast_table", CastTable))
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', 'int main(void) {']
    for cname, cls in structs:
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    src = tmp_path / "off.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "off"
    subprocess.run([cc, "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {}
    for line in out:
        if line:
            a, b, c = line.split()
            got[(a, b)] = int(c)
    for cname, cls in structs:
        assert got[(cname, "size")] == ctypes.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert got[(cname, fname)] == getattr(cls, fname).offset, (cname, fname)


def test_error_path_without_gpu():
    """A bad argument is rejected before any device work, with a message."""
    from transmil_deepgraft_amd import _lib
    with pytest.raises(RuntimeError, match="n must be a positive multiple of 256"):
        _lib.call("tm_nys_landmarks", 1, None, None, 8, 100, None, None, None, None, None)
    assert "multiple of 256" in _lib.last_error()


def test_build_info():
    from transmil_deepgraft_amd import _lib
    assert b"gfx950" in _lib.lib().tm_build_info()


def test_product_library_has_no_diagnostic_switches():
    """Kernel-variant switches and timing stamps live only in the TM_DIAG build
    (libtransmil_hip_diag.so, scripts/microbench.py): the product library exports no tm_debug_*
    entry point, so no process-global state can change another stream's kernels."""
    import subprocess
    from transmil_deepgraft_amd import _lib
    lib = _lib.lib()
    for name in _lib.DIAG_SIGS:
        assert not hasattr(lib, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True)
    if nm.returncode == 0:
        assert "tm_debug" not in nm.stdout
