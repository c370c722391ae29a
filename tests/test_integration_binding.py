"""The Rust binding INTEGRATION.md §2 shows a maintainer (src/rps_ffi.rs) agrees with
include/rps.h, checked without rustc (there is none in this image):

* every `#[repr(C)]` struct has the C struct's size and field offsets (Rust repr(C) lays out
  fields like C; the C side is compiled here with gcc and printed with offsetof);
* the `extern "C"` block declares every function of the header, with the same number of
  parameters and the same parameter / return classes (pointer, 32-bit integer, 64-bit
  integer, f32, f64)."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "rps.h")
DOC = os.path.join(ROOT, "INTEGRATION.md")

# Rust struct -> C typedef (the reference's own types map to rps_particle / rps_config)
STRUCTS = {"rps_attractor": "rps_attractor", "rps_ext_config": "rps_ext_config",
           "rps_create_info": "rps_create_info", "rps_stats": "rps_stats", "rps_sph_cost": "rps_sph_cost"}
RUST_SCALARS = {"u8": (1, "i"), "i8": (1, "i"), "u16": (2, "i"), "i16": (2, "i"), "u32": (4, "i"),
                "i32": (4, "i"), "c_int": (4, "i"), "u64": (8, "i"), "i64": (8, "i"), "usize": (8, "i"),
                "f32": (4, "f"), "f64": (8, "d")}


def rust_block():
    src = open(DOC).read()
    m = re.search(r"```rust\n(.*?)```", src, re.S)
    assert m, "INTEGRATION.md has no rust block"
    return re.sub(r"//[^\n]*", "", m.group(1))


def rust_structs(code):
    out = {}
    for name, body in re.findall(r"#\[repr\(C\)\][^\n]*\n?\s*pub struct (\w+)\s*\{(.*?)\}", code, re.S):
        fields = [(f, t.strip()) for f, t in re.findall(r"pub (\w+)\s*:\s*([^,]+?)\s*(?:,|$)", body.strip(), re.S)]
        out[name] = fields
    return out


def rust_layout(structs, name):
    """(size, align, {field: offset}) with C / repr(C) rules."""
    off, align, offs = 0, 1, {}
    for f, t in structs[name]:
        size, al = rust_type_size(structs, t)
        off = (off + al - 1) // al * al
        offs[f] = off
        off += size
        align = max(align, al)
    return (off + align - 1) // align * align, align, offs


def rust_type_size(structs, t):
    t = t.strip()
    m = re.fullmatch(r"\[(.+);\s*(\d+)\]", t)
    if m:
        size, al = rust_type_size(structs, m.group(1))
        return size * int(m.group(2)), al
    if t in RUST_SCALARS:
        s = RUST_SCALARS[t][0]
        return s, s
    if t.startswith("*"):
        return 8, 8
    if t in structs:
        size, al, _ = rust_layout(structs, t)
        return size, al
    raise AssertionError(f"unknown Rust field type {t}")


@pytest.fixture(scope="module")
def c_layouts(tmp_path_factory):
    code = rust_block()
    structs = rust_structs(code)
    lines = ['#include "rps.h"', "#include <stdio.h>", "#include <stddef.h>", "int main(void){"]
    for rs, cs in STRUCTS.items():
        lines.append(f'printf("{cs} size %zu\\n", sizeof({cs}));')
        for f, _ in structs[rs]:
            lines.append(f'printf("{cs} {f} %zu\\n", offsetof({cs}, {f}));')
    lines.append("return 0;}")
    d = tmp_path_factory.mktemp("layout")
    (d / "l.c").write_text("\n".join(lines) + "\n")
    subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), "-o", str(d / "l"), str(d / "l.c")], check=True)
    out = subprocess.run([str(d / "l")], capture_output=True, text=True, check=True).stdout
    res = {}
    for line in out.splitlines():
        s, f, v = line.split()
        res[(s, f)] = int(v)
    return structs, res


def test_rust_structs_match_c_layout(c_layouts):
    structs, c = c_layouts
    assert set(STRUCTS) <= set(structs), sorted(structs)
    for rs, cs in STRUCTS.items():
        size, _, offs = rust_layout(structs, rs)
        assert size == c[(cs, "size")], (rs, size, c[(cs, "size")])
        for f, o in offs.items():
            assert o == c[(cs, f)], (rs, f, o, c[(cs, f)])


def c_prototypes():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for ret, name, args in re.findall(r"\n\s*((?:const\s+)?[\w]+\s*\**)\s*(rps_\w+)\s*\(([^)]*)\)\s*;", src):
        params = [] if args.strip() in ("", "void") else [a.strip() for a in args.split(",")]
        out[name] = (ret.strip(), params)
    return out


def c_class(decl):
    if "*" in decl:
        return "p"
    base = re.sub(r"\b(const|unsigned|signed)\b", "", decl).split()
    t = base[0] if base else decl
    return {"uint64_t": "i8", "int64_t": "i8", "size_t": "i8", "uint32_t": "i4", "int32_t": "i4", "int": "i4",
            "float": "f4", "double": "f8", "void": "v"}[t]


def rust_class(t):
    t = t.strip()
    if t.startswith("*") or t.startswith("&"):
        return "p"
    if t in RUST_SCALARS:
        size, kind = RUST_SCALARS[t]
        return {"i": "i", "f": "f", "d": "f"}[kind] + str(size)
    raise AssertionError(f"unknown Rust parameter type {t}")


def rust_fns():
    code = rust_block()
    ext = re.search(r'extern "C"\s*\{(.*?)\n\}', code, re.S).group(1)
    out = {}
    for name, args, ret in re.findall(r"pub fn (rps_\w+)\(([^)]*)\)\s*(?:->\s*([^;]+))?;", ext):
        params = [a.split(":", 1)[1].strip() for a in args.split(",") if a.strip()]
        out[name] = (ret.strip() if ret else "()", params)
    return out


def test_rust_extern_block_matches_header():
    from test_abi import declared_functions

    c = c_prototypes()
    assert sorted(c) == declared_functions()  # the prototype parser saw every declaration
    r = rust_fns()
    assert set(c) == set(r), {"not bound in INTEGRATION.md": sorted(set(c) - set(r)),
                              "not in rps.h": sorted(set(r) - set(c))}
    for name, (cret, cparams) in c.items():
        rret, rparams = r[name]
        assert len(cparams) == len(rparams), name
        for cp, rp in zip(cparams, rparams):
            assert c_class(cp) == rust_class(rp), (name, cp, rp)
        assert (c_class(cret) if cret != "void" else "v") == (rust_class(rret) if rret != "()" else "v"), name
