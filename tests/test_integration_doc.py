"""INTEGRATION.md's Rust binding against include/cdb_merge.h (no Rust toolchain here, so the binding is
checked as text): every cdb_* function the header declares is bound and nothing else is, and every
`size_of::<T>() == N` the Rust block asserts equals the C sizeof of T, compiled with the system C
compiler against the header. A header change that a binding would silently misread fails here."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rust_block():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    start = text.index("## 2. The binding")
    block = text[start:text.index("## 3.", start)]
    m = re.search(r"```rust\n(.*?)```", block, re.S)
    assert m, "no rust block in INTEGRATION.md section 2"
    return m.group(1)


def _header_functions():
    text = open(os.path.join(ROOT, "include", "cdb_merge.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(cdb_\w+)\s*\(", text))


def test_binding_declares_every_header_function():
    rust = _rust_block()
    bound = set(re.findall(r"pub fn (cdb_\w+)\s*\(", rust))
    header = _header_functions()
    assert header - bound == set(), f"header functions missing from the Rust binding: {sorted(header - bound)}"
    assert bound - header == set(), f"Rust binding names functions the header does not declare: {sorted(bound - header)}"


def test_binding_struct_sizes_match_c(tmp_path):
    rust = _rust_block()
    sizes = dict(re.findall(r"size_of::<(cdb_\w+)>\(\) == (\d+)", rust))
    structs = set(re.findall(r"pub struct (cdb_\w+) \{", rust))
    opaque = {"cdb_ctx", "cdb_batch", "cdb_merged", "cdb_ops"}
    assert structs - opaque - set(sizes) == set(), f"structs without a size assert: {structs - opaque - set(sizes)}"
    src = tmp_path / "sizes.c"
    src.write_text('#include <stdio.h>\n#include "cdb_merge.h"\nint main(void) {\n' +
                   "".join(f'  printf("{n} %zu\\n", sizeof({n}));\n' for n in sorted(sizes)) + "  return 0;\n}\n")
    exe = tmp_path / "sizes"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    out = subprocess.check_output([str(exe)], text=True)
    got = dict(line.split() for line in out.strip().splitlines())
    for n, v in sizes.items():
        assert got[n] == v, f"sizeof({n}) = {got[n]} in C, INTEGRATION.md asserts {v}"


def test_binding_sizes_match_abi_pins():
    """The same numbers as tests/abi/abi_check.c's compile-time PIN_SIZEs."""
    rust = dict(re.findall(r"size_of::<(cdb_\w+)>\(\) == (\d+)", _rust_block()))
    pins = dict(re.findall(r"PIN_SIZE\((cdb_\w+), (\d+)\)", open(os.path.join(ROOT, "tests", "abi", "abi_check.c")).read()))
    for n, v in pins.items():
        assert rust.get(n) == v, f"abi_check.c pins sizeof({n}) = {v}, INTEGRATION.md asserts {rust.get(n)}"
