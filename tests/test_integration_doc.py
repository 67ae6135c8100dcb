"""INTEGRATION.md's C-ABI examples agree with include/eloqstore_pcs.h.

VERDICT r02 weak #7: a ctypes example that passes fewer arguments than the
prototype leaves the trailing `flags` word to whatever is on the stack, which
can switch verification off.  Every `pcs_*(...)` call in every fenced block of
INTEGRATION.md (C, C++, Python, Go) and every ctypes `argtypes` list is
counted against the header prototype; `compile-c:` blocks are compiled as C11.
No GPU and no reference tree needed.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOC = os.path.join(ROOT, "INTEGRATION.md")
HEADER = os.path.join(ROOT, "include", "eloqstore_pcs.h")

_FENCE = re.compile(r"```(\w+)\n(.*?)\n```", re.S)
_PROTO = re.compile(r"\b(pcs_\w+)\s*\(([^;{]*?)\)\s*;", re.S)
_CALL = re.compile(r"\b(pcs_\w+)\s*\(")
_ARGTYPES = re.compile(r"\.(pcs_\w+)\.argtypes\s*=\s*(?:\w+\.(pcs_\w+)\.argtypes\s*\+\s*)?\[(.*?)\]", re.S)


def header_arity() -> dict:
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for name, params in _PROTO.findall(text):
        params = " ".join(params.split())
        out[name] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def _split_args(text: str, start: int):
    """Top-level argument count of the call whose '(' is at text[start]."""
    depth, n, has_arg = 0, 0, False
    for i in range(start, len(text)):
        c = text[i]
        if c in "([{":
            depth += 1
            if depth == 1:
                continue
        elif c in ")]}":
            depth -= 1
            if depth == 0:
                return n + (1 if has_arg else 0)
        if depth == 1:
            if c == ",":
                n += 1
                has_arg = False
            elif not c.isspace():
                has_arg = True
    raise ValueError("unbalanced call")


def check_block(lang: str, body: str, arity: dict) -> list:
    errors = []
    for m in _CALL.finditer(body):
        name = m.group(1)
        if name not in arity:
            errors.append(f"{lang}: {name} is not declared in eloqstore_pcs.h")
            continue
        got = _split_args(body, m.end() - 1)
        if got != arity[name]:
            errors.append(f"{lang}: {name} called with {got} arguments, header declares {arity[name]}")
    for name, base, items in _ARGTYPES.findall(body):
        n = len([x for x in items.split(",") if x.strip()]) + (arity.get(base, 0) if base else 0)
        if name not in arity or n != arity[name]:
            errors.append(f"{lang}: {name}.argtypes has {n} entries, header declares {arity.get(name)}")
    return errors


def doc_blocks():
    return _FENCE.findall(open(DOC).read())


def test_header_prototypes_parse():
    a = header_arity()
    assert a["pcs_pages_validate_host"] == 6 and a["pcs_pages_validate_host_ex"] == 7
    assert a["pcs_batch_submit"] == 6 and a["pcs_batch_submit_ex"] == 7
    assert a["pcs_version"] == 0 and len(a) >= 30


def test_every_pcs_call_in_the_doc_matches_the_header():
    arity = header_arity()
    blocks = doc_blocks()
    langs = {lang for lang, _ in blocks}
    assert {"python", "go", "c", "cpp"} <= langs
    calls = sum(len(_CALL.findall(body)) for _, body in blocks)
    assert calls >= 5
    errors = [e for lang, body in blocks for e in check_block(lang, body, arity)]
    assert not errors, "\n".join(errors)


def test_checker_catches_the_round2_mistakes():
    """Negative controls: the shapes of the mistakes VERDICT r02 found."""
    arity = header_arity()
    bad_py = ("lib.pcs_pages_validate_host_ex.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,\n"
              "    ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]\n"
              "rc = lib.pcs_pages_validate_host_ex(page_ptr_array, 4096, n, 0, ok_buf, ctypes.byref(first_bad))\n")
    errs = check_block("python", bad_py, arity)
    assert len(errs) == 2 and all("pcs_pages_validate_host_ex" in e for e in errs)
    bad_go = "rc := C.pcs_batch_submit(b, C.PCS_BATCH_VALIDATE, &p[0], 4096, C.uint64_t(n), 0, f(x, y))"
    assert check_block("go", bad_go, arity) == [
        "go: pcs_batch_submit called with 7 arguments, header declares 6"]


_C_BLOCK = re.compile(r"<!-- compile-c: (\w+) -->\s*\n```c\n(.*?)\n```", re.S)


@pytest.mark.parametrize("name,body", _C_BLOCK.findall(open(DOC).read()))
def test_c_blocks_compile(name, body, tmp_path):
    src = tmp_path / f"{name}.c"
    src.write_text(body + "\n")
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-c", f"-I{ROOT}/include", str(src),
                        "-o", str(tmp_path / f"{name}.o")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    nm = subprocess.run(["nm", "-u", str(tmp_path / f"{name}.o")], capture_output=True, text=True).stdout
    assert "pcs_" in nm


def test_doc_has_a_c_block():
    assert _C_BLOCK.findall(open(DOC).read())
