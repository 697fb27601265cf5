"""The C-ABI boundary (include/lsr.h) on CPU: liblsr.so loads, exports every
entry point the header declares, the ctypes mirrors in langsplatv2_amd/_lib.py
have the C header's exact layout, and the host-only entry points answer.
No compute entry point is called here (there is no GPU in this container)."""
import ctypes
import os
import re
import subprocess

import pytest

from langsplatv2_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lsr.h")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "langsplatv2_amd", "csrc")], check=True,
                       timeout=1800)
    return _lib.load()


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    names = set(re.findall(r"^[A-Za-z_][\w \*]*?\b(lsr_\w+)\s*\(", src, flags=re.M))
    names.discard("lsr_alloc_fn")
    return sorted(names)


def test_header_declares_the_bound_entry_points():
    assert set(header_functions()) == set(_lib.EXPORTS)


def test_library_exports_every_header_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    for name in header_functions():
        assert name in exported, name
        assert hasattr(lib, name)


def test_host_only_entry_points(lib):
    assert lib.lsr_abi_version() >= 1
    assert lib.lsr_max_lang_dim() >= 64
    assert lib.lsr_strerror(0).decode().lower() in ("ok", "success", "no error")
    for code in range(1, 8):
        assert isinstance(lib.lsr_strerror(code), bytes)
    # argument validation happens before any device call
    assert lib.lsr_topk_code_forward(None, 10, 1, 48, 4, None, None, None, 0, 0, None) == 2  # K % 64 -> unsupported
    assert lib.lsr_topk_code_forward(None, 10, 1, 64, 0, None, None, None, 0, 0, None) == 1  # k < 1
    assert lib.lsr_topk_code_forward(1, 10, 1, 64, 4, None, None, None, 0, 0, None) == 1     # no output
    assert lib.lsr_topk_code_forward(None, 0, 1, 64, 4, 1, None, None, 0, 0, None) == 0      # N = 0: no-op
    assert lib.lsr_topk_code_backward(None, None, 10, 1, 64, 65, None, None) == 1           # k > K


def _c_layout(structs):
    """sizeof/offsetof of each (C struct, ctypes mirror) pair, from gcc."""
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void) {"]
    for cname, cls in structs:
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines += ["return 0; }"]
    return "\n".join(lines)


def _check_layout(tmp_path, structs, header_dir):
    c = tmp_path / "layout.c"
    c.write_text(_c_layout(structs))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", header_dir, str(c), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    got = {(a, b): int(v) for a, b, v in (ln.split() for ln in out if ln)}
    for cname, cls in structs:
        assert got[(cname, "sizeof")] == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert got[(cname, f)] == getattr(cls, f).offset, (cname, f)


def test_ctypes_structs_match_c_header(tmp_path):
    structs = [("lsr_settings", _lib.Settings), ("lsr_inputs", _lib.Inputs), ("lsr_fwd_out", _lib.FwdOut),
               ("lsr_bwd_in", _lib.BwdIn), ("lsr_bwd_out", _lib.BwdOut)]
    _check_layout(tmp_path, structs, os.path.dirname(HEADER))


def test_oracle_structs_match_oracle_header(tmp_path):
    import oracle.oracle as O
    global HEADER
    saved = HEADER
    HEADER = os.path.join(ROOT, "oracle", "lsr_oracle.h")
    try:
        structs = [("lso_settings", O._Settings), ("lso_inputs", O._Inputs), ("lso_geom", O._Geom),
                   ("lso_render_grads", O._RGrads), ("lso_param_grads", O._PGrads)]
        _check_layout(tmp_path, structs, os.path.dirname(HEADER))
    finally:
        HEADER = saved


def test_product_path_does_not_reference_the_oracle():
    """The shipped package must never import / link the oracle."""
    for dirpath, _, files in (w for pkg in ("langsplatv2_amd", "diff_gaussian_rasterization", "simple_knn")
                              for w in os.walk(os.path.join(ROOT, pkg))):
        if "_build" in dirpath:
            continue
        for fn in files:
            if fn.endswith((".py", ".hip", ".h", ".cpp", "Makefile")):
                txt = open(os.path.join(dirpath, fn)).read()
                assert not re.search(r'#include\s*[<"][^>"]*oracle', txt), fn
                assert not re.search(r"^\s*(import oracle|from oracle)", txt, flags=re.M), fn
                assert "liblsr_oracle" not in txt and "-llsr_oracle" not in txt, fn
    assert "oracle" not in subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout \
        if os.path.exists(_lib.LIB_PATH) else True
