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


def _prototypes():
    """name -> parameter count of every prototype in the header (comments stripped)."""
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(tm_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_ctypes_arity_matches_header():
    """Every ctypes argtypes list has exactly as many entries as the C prototype has parameters
    (a signature change in the header without the binding would pass garbage for the stream)."""
    from transmil_deepgraft_amd import _lib
    protos = _prototypes()
    bad = {n: (len(args), protos.get(n)) for n, (_, args) in _lib._SIGS.items() if protos.get(n) != len(args)}
    assert not bad, bad


def test_reduce_queue_is_caller_owned():
    """The deferral queue is a caller-owned host object: two queues are independent, appending
    needs no GPU (no launch happens until tm_reduce_flush), an invalid handle is refused, and the
    reduction entry points take the queue explicitly (reentrant across streams)."""
    import ctypes as C
    from transmil_deepgraft_amd import _lib
    lib = _lib.lib()
    assert not hasattr(lib, "tm_reduce_defer")        # the old process-global switch is gone
    qa, qb = C.c_void_p(lib.tm_reduce_queue_create()), C.c_void_p(lib.tm_reduce_queue_create())
    assert qa.value and qb.value and qa.value != qb.value
    try:
        assert lib.tm_reduce_queue_pending(qa) == 0 and lib.tm_reduce_queue_pending(qb) == 0
        slab, out = C.c_void_p(0x10000), C.c_void_p(0x20000)      # never dereferenced on the host
        for i in range(3):
            _lib.call("tm_splitk_reduce", slab, out, 4, 1024, C.c_float(1.0), 0, qa, None)
        _lib.call("tm_splitk_reduce", slab, out, 4, 0, C.c_float(1.0), 0, qb, None)   # empty: not queued
        assert lib.tm_reduce_queue_pending(qa) == 3
        assert lib.tm_reduce_queue_pending(qb) == 0
        _lib.call("tm_reduce_flush", qb, None)              # nothing queued: no launch
        with pytest.raises(RuntimeError, match="not a tm_reduce_queue"):
            _lib.call("tm_reduce_flush", None, None)
        assert lib.tm_reduce_queue_pending(None) == -1
    finally:
        lib.tm_reduce_queue_destroy(qa)
        lib.tm_reduce_queue_destroy(qb)


def test_engine_binds_one_queue_per_backward_call_and_thread():
    """engine.reduce_scope binds a fresh queue per call on the calling thread only; the call
    sites pass it only inside defer_reductions()."""
    import threading
    from transmil_deepgraft_amd import engine as E
    assert E._rq().value is None
    seen = {}

    def worker(i):
        with E.reduce_scope() as q:
            with E.defer_reductions():
                seen[i] = (q.handle.value, E._rq().value)
            seen[(i, "after")] = E._rq().value

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    with E.reduce_scope() as outer:
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert E._rq().value is None                  # bound but not deferring here
        with E.defer_reductions():
            assert E._rq().value == outer.handle.value
    assert seen[0][0] == seen[0][1] and seen[1][0] == seen[1][1]
    assert seen[(0, "after")] is None and seen[(1, "after")] is None
    assert E._rq().value is None


def _strip_diag_blocks(text):
    """The source without `#ifdef TM_DIAG ... #endif` blocks (the diagnostic build's code)."""
    out, depth, diag = [], 0, []
    for line in text.split("\n"):
        s = line.strip()
        if s.startswith("#if"):
            depth += 1
            diag.append(s.startswith("#ifdef TM_DIAG") or s.startswith("#if defined(TM_DIAG)"))
            continue
        if s.startswith("#endif"):
            depth -= 1
            diag.pop()
            continue
        if s.startswith("#else") and diag:
            diag[-1] = not diag[-1] if diag[-1] else diag[-1]
            continue
        if not any(diag):
            out.append(line)
    return "\n".join(out)


def test_only_the_documented_entry_point_synchronises():
    """The header promises no host synchronisation and no library-owned device scratch, with ONE
    documented exception: tm_conv1x1_tune (host-timed hipBLASLt algorithm search, refused during
    capture).  No product source waits on the device or allocates device memory anywhere else
    (TM_DIAG-only code excluded: the diagnostic library is not the product)."""
    import glob
    head = open(HEADER).read()
    conventions = head[:head.index("#ifndef TRANSMIL_HIP_H")]
    assert "ONE documented" in conventions and "tm_conv1x1_tune" in conventions
    proto = head[head.index("int tm_conv1x1_tune("):]
    assert "refused" in head[head.index("THE EXCEPTION"):head.index("int tm_conv1x1_tune(")]
    assert proto
    pat = re.compile(r"\b(hipDeviceSynchronize|hipStreamSynchronize|hipEventSynchronize|hipMemcpy|"
                     r"hipMemcpyFromSymbol|hipMalloc|hipMallocManaged|hipHostMalloc)\s*\(")
    hits = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "transmil_deepgraft_amd", "csrc", "*.hip")) +
                       glob.glob(os.path.join(ROOT, "transmil_deepgraft_amd", "csrc", "*.h"))):
        text = _strip_diag_blocks(open(path).read())
        found = pat.findall(text)
        if found:
            hits[os.path.basename(path)] = found
    assert hits == {"conv1x1.hip": ["hipEventSynchronize"]}, hits
    src = open(os.path.join(ROOT, "transmil_deepgraft_amd", "csrc", "conv1x1.hip")).read()
    # ... and that one wait sits in the tuning branch, which refuses a capturing stream
    assert src.index("hipEventSynchronize") > src.index("if (tune && !p->tuned)")
    assert "not during stream capture" in src
