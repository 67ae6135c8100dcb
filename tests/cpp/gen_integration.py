"""Compile INTEGRATION.md's call-site snippets against the reference's page.h.

TEST INFRASTRUCTURE.  Every fenced ```cpp block preceded by a
`<!-- compile: NAME -->` line in INTEGRATION.md is pasted verbatim into
tests/cpp/integration_harness.cpp.in at @SNIPPET(NAME)@; the translation unit
includes the reference's own include/storage/page.h (read in place from
/root/reference, never copied) next to include/eloqstore/page_checksum.h and
links libeloqstore_pcs.so (+ the CPU oracle as checker).

    python tests/cpp/gen_integration.py [--syntax-only] [--out BINARY]

The binary (default tests/cpp/integration_snippets, git-ignored) travels to
the GPU box, where tests/test_gpu_integration.py runs it.
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = os.environ.get("ELOQSTORE_REFERENCE", "/root/reference")
TEMPLATE = os.path.join(ROOT, "tests", "cpp", "integration_harness.cpp.in")
DOC = os.path.join(ROOT, "INTEGRATION.md")
DEFAULT_OUT = os.path.join(ROOT, "tests", "cpp", "integration_snippets")

_BLOCK = re.compile(r"<!-- compile: (\w+) -->\s*\n```cpp\n(.*?)\n```", re.S)
_MARK = re.compile(r"^([ \t]*)@SNIPPET\((\w+)\)@[ \t]*$", re.M)


def snippets(doc_text: str) -> dict[str, str]:
    out: dict[str, str] = {}
    for name, body in _BLOCK.findall(doc_text):
        if name in out:
            raise ValueError(f"snippet {name!r} appears twice in INTEGRATION.md")
        out[name] = body
    return out


def render(doc_text: str, template_text: str) -> str:
    blocks = snippets(doc_text)
    wanted = {m.group(2) for m in _MARK.finditer(template_text)}
    missing = wanted - blocks.keys()
    unused = blocks.keys() - wanted
    if missing or unused:
        raise ValueError(f"snippet mismatch: missing in doc {sorted(missing)}, unused {sorted(unused)}")

    def paste(m: re.Match) -> str:
        indent, name = m.group(1), m.group(2)
        body = "\n".join((indent + line) if line.strip() else "" for line in blocks[name].splitlines())
        return f"{indent}// ---- INTEGRATION.md snippet: {name} ----\n{body}"

    return _MARK.sub(paste, template_text)


def reference_present() -> bool:
    return os.path.isfile(os.path.join(REF, "include", "storage", "page.h"))


def compile_tu(out: str, syntax_only: bool = False) -> subprocess.CompletedProcess:
    src = render(open(DOC).read(), open(TEMPLATE).read())
    build = os.path.join(ROOT, "eloqstore_amd", "build")
    os.makedirs(build, exist_ok=True)
    tu = os.path.join(build, "integration_snippets.cpp")
    with open(tu, "w") as f:
        f.write(src)
    cmd = ["g++", "-std=c++20", "-O1", "-Wall", "-Wno-unused-variable",
           f"-I{REF}/include", f"-I{REF}", f"-I{ROOT}/include", f"-I{ROOT}/oracle", tu]
    if syntax_only:
        cmd.append("-fsyntax-only")
    else:
        lib = os.path.join(ROOT, "eloqstore_amd")
        orc = os.path.join(ROOT, "oracle")
        # page.cpp's CPU SetChecksum/ValidateChecksum stand-ins hash with the
        # reference's own xxhash.c (oracle/_ref, built by `make -C oracle ref`)
        cmd += ["-o", out, f"-L{lib}", "-leloqstore_pcs", f"-L{orc}", "-loracle", f"-L{orc}/_ref", "-lxxhash_ref",
                "-Wl,-rpath-link,/opt/rocm/lib",
                "-Wl,-rpath,$ORIGIN/../../eloqstore_amd", "-Wl,-rpath,$ORIGIN/../../oracle",
                "-Wl,-rpath,$ORIGIN/../../oracle/_ref"]
    return subprocess.run(cmd, capture_output=True, text=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--syntax-only", action="store_true")
    ap.add_argument("--out", default=DEFAULT_OUT)
    a = ap.parse_args()
    if not reference_present():
        print(f"reference tree absent ({REF}): integration snippets not compiled")
        return 0
    r = compile_tu(a.out, a.syntax_only)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr)
    if r.returncode == 0:
        print("integration snippets compiled" + ("" if a.syntax_only else f" -> {a.out}"))
    return r.returncode


if __name__ == "__main__":
    sys.exit(main())
