"""The reference-side Rust binding shown in INTEGRATION.md against the C ABI.

No rustc exists here, so the binding a maintainer would paste into the
reference crate (`src/amd.rs`) cannot be compiled.  This
test checks it against the header instead, field for field:

* every `#[repr(C)]` struct of the Rust snippet is laid out with Rust's
  repr(C) rules (each field at the next multiple of its alignment, the size
  rounded up to the largest alignment) and compared with a C probe compiled
  from include/raytrace_amd.h with gcc (sizeof / offsetof of every field the
  header declares): same field names in the same order, same scalar types,
  same offsets, same size.  A field added on either side fails the test;
* every `pub const` equals the header's macro / enum value;
* every `extern "C"` function exists in the header with the same number of
  parameters, and the library exports it;
* rt_abi_version() returns the header's RT_ABI_VERSION.

Replaces nothing in the reference (it has no FFI); guards INTEGRATION.md §2.
"""
import os
import re
import shutil
import subprocess

import pytest

import libraytrace as lr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "raytrace_amd.h")
DOC = os.path.join(ROOT, "INTEGRATION.md")

# Rust scalar type -> (C type the header must use, size = alignment)
RUST_SCALARS = {"u8": ("uint8_t", 1), "i8": ("int8_t", 1), "u16": ("uint16_t", 2), "i16": ("int16_t", 2),
                "u32": ("uint32_t", 4), "i32": ("int32_t", 4), "f32": ("float", 4), "c_int": ("int", 4),
                "c_uint": ("unsigned", 4), "u64": ("uint64_t", 8), "i64": ("int64_t", 8), "f64": ("double", 8),
                "usize": ("size_t", 8)}


def _strip_c_comments(text):
    return re.sub(r"//[^\n]*", "", re.sub(r"/\*.*?\*/", "", text, flags=re.S))


def _rust_blocks():
    text = open(DOC).read()
    return "\n".join(re.findall(r"```rust\n(.*?)```", text, flags=re.S))


def rust_structs():
    """{RustName: [(field, scalar, count)]} for every #[repr(C)] struct with fields."""
    src = re.sub(r"//[^\n]*", "", _rust_blocks())
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\][^{;]*?pub struct (\w+)\s*\{(.*?)\}", src, flags=re.S):
        name, body = m.group(1), m.group(2)
        fields = []
        for fm in re.finditer(r"pub (\w+)\s*:\s*(\[\s*(\w+)\s*;\s*(\d+)\s*\]|\w+)", body):
            if fm.group(3):
                fields.append((fm.group(1), fm.group(3), int(fm.group(4))))
            else:
                fields.append((fm.group(1), fm.group(2), 1))
        if fields and not (len(fields) == 1 and fields[0][0] == "_p"):
            out[name] = fields
    return out


def rust_consts():
    return {m.group(1): int(m.group(2)) for m in
            re.finditer(r"pub const (\w+)\s*:\s*\w+\s*=\s*(-?\d+)\s*;", _rust_blocks())}


def rust_functions():
    src = re.sub(r"//[^\n]*", "", _rust_blocks())
    out = {}
    for blk in re.findall(r'extern "C"\s*\{(.*?)\n\}', src, flags=re.S):
        for m in re.finditer(r"pub fn (\w+)\s*\((.*?)\)", blk, flags=re.S):
            args = [a for a in m.group(2).split(",") if a.strip()]
            out[m.group(1)] = len(args)
    return out


def snake(name):
    return re.sub(r"(?<!^)([A-Z])", r"_\1", name).lower()      # RtRenderOpts -> rt_render_opts


def c_struct_fields(cname):
    """[(ctype, field, count)] of `typedef struct { ... } cname;` in the header."""
    text = _strip_c_comments(open(HEADER).read())
    m = re.search(r"typedef struct\s*\{([^{}]*)\}\s*" + cname + r"\s*;", text)
    assert m, f"{cname} not found in the header"
    fields = []
    for decl in m.group(1).split(";"):
        decl = " ".join(decl.split())
        if not decl:
            continue
        dm = re.match(r"((?:const\s+)?[\w]+(?:\s*\*)?)\s+(.*)", decl)
        ctype, names = dm.group(1), dm.group(2)
        for nm in names.split(","):
            nm = nm.strip()
            am = re.match(r"(\w+)\s*\[\s*(\d+)\s*\]", nm)
            fields.append((ctype, am.group(1), int(am.group(2))) if am else (ctype, nm, 1))
    return fields


def header_constants():
    text = _strip_c_comments(open(HEADER).read())
    out = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define (RT_\w+)\s+(-?\d+)", text)}
    for m in re.finditer(r"\b(RT_\w+)\s*=\s*(-?\d+)", text):
        out[m.group(1)] = int(m.group(2))
    return out


def header_function_arity():
    text = _strip_c_comments(open(HEADER).read())
    out = {}
    for m in re.finditer(r"\b(rt_\w+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else len(args.split(","))
    return out


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    """{cname: (sizeof, {field: (offset, sizeof)})} from a gcc-compiled probe of the header."""
    cc = shutil.which("gcc") or shutil.which("cc")
    if not cc:
        pytest.skip("no C compiler")
    names = [snake(n) for n in rust_structs()]
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname in names:
        lines.append(f'printf("S {cname} %zu\\n", sizeof({cname}));')
        for _, f, _ in c_struct_fields(cname):
            lines.append(f'printf("F {cname} {f} %zu %zu\\n", offsetof({cname}, {f}), sizeof((({cname}*)0)->{f}));')
    lines.append("return 0; }")
    d = tmp_path_factory.mktemp("abi_probe")
    src, exe = d / "probe.c", d / "probe"
    src.write_text("\n".join(lines))
    subprocess.run([cc, "-std=c11", "-Wall", "-o", str(exe), str(src)], check=True)
    out = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        p = line.split()
        if p[0] == "S":
            out.setdefault(p[1], [0, {}])[0] = int(p[2])
        else:
            out.setdefault(p[1], [0, {}])[1][p[2]] = (int(p[3]), int(p[4]))
    return out


def test_binding_declares_the_structs_the_pixel_loop_passes():
    rs = rust_structs()
    assert {"RtRenderOpts", "RtStats"} <= set(rs), sorted(rs)


def test_rust_structs_match_the_header_field_for_field(c_layout):
    for rname, rfields in rust_structs().items():
        cname = snake(rname)
        cfields = c_struct_fields(cname)
        assert [f for f, _, _ in rfields] == [f for _, f, _ in cfields], f"{rname} vs {cname}: field names/order"
        size, offs = c_layout[cname]
        off, align = 0, 1
        for (fname, rty, cnt), (cty, _, ccnt) in zip(rfields, cfields):
            assert rty in RUST_SCALARS, f"{rname}.{fname}: unsupported Rust type {rty}"
            want_c, sz = RUST_SCALARS[rty]
            assert cty == want_c, f"{rname}.{fname}: Rust {rty} but the header says {cty}"
            assert cnt == ccnt, f"{rname}.{fname}: array length {cnt} vs {ccnt}"
            off = (off + sz - 1) // sz * sz                       # repr(C): aligned to the scalar's size
            assert offs[fname] == (off, sz * cnt), f"{rname}.{fname}: Rust offset {off} vs C {offs[fname]}"
            off += sz * cnt
            align = max(align, sz)
        rsize = (off + align - 1) // align * align
        assert rsize == size, f"{rname}: Rust size {rsize} vs sizeof({cname}) = {size}"


def test_abi_sizes_at_version_5(c_layout):
    assert c_layout["rt_render_opts"][0] == 72
    assert c_layout["rt_stats"][0] == 80


def test_rust_constants_match_the_header():
    hc = header_constants()
    rc = rust_consts()
    assert "RT_ABI_VERSION" in rc
    for k, v in rc.items():
        assert hc.get(k) == v, f"{k}: Rust {v}, header {hc.get(k)}"


def test_rust_functions_exist_with_the_same_arity():
    hf = header_function_arity()
    rf = rust_functions()
    assert "rt_render" in rf and "rt_abi_version" in rf
    for name, n in rf.items():
        assert name in hf, f"{name} is not declared in the header"
        assert hf[name] == n, f"{name}: Rust binds {n} parameters, the header declares {hf[name]}"
        assert hasattr(lr.lib, name), f"{name} is not exported by librtamd.so"


def test_library_reports_the_header_abi_version():
    assert lr.lib.rt_abi_version() == header_constants()["RT_ABI_VERSION"] == lr.RT_ABI_VERSION


def test_a_field_added_on_either_side_is_caught(c_layout):
    """The checker itself: an extra Rust field or a missing one changes the verdict."""
    rs = rust_structs()["RtStats"]
    cf = [f for _, f, _ in c_struct_fields("rt_stats")]
    assert [f for f, _, _ in rs] == cf
    assert [f for f, _, _ in rs[:-1]] != cf and [f for f, _, _ in rs] + ["extra"] != cf
