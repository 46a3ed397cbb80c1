"""The Rust FFI crate rust/gossipsim-sys (the binding north_star names for
rust-test-node) against the C header it declares: no cargo
in this container, so its src/lib.rs is parsed here and every #[repr(C)]
struct's field order, names and widths, the ABI version and every extern fn's
name and arity are checked against include/gossipsim.h."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gossipsim.h")
LIBRS = os.path.join(ROOT, "rust", "gossipsim-sys", "src", "lib.rs")
STRUCTS = ["gs_config", "gs_publish", "gs_msg_summary", "gs_result_sink", "gs_stats", "gs_injector",
           "gs_part_record"]

C_TYPES = {"uint64_t": "u64", "uint32_t": "u32", "int32_t": "i32", "uint8_t": "u8", "double": "f64",
           "gs_block_fn": "fnptr", "gs_lat_fn": "fnptr"}
R_TYPES = {"u64": "u64", "u32": "u32", "i32": "i32", "u8": "u8", "f64": "f64", "gs_block_fn": "fnptr",
           "gs_lat_fn": "fnptr"}


def _strip_c(src):
    return re.sub(r"//[^\n]*", "", re.sub(r"/\*.*?\*/", "", src, flags=re.S))


def _header():
    return _strip_c(open(HEADER).read())


def _consts(src):
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"#define\s+(\w+)\s+(\d+)u?\b", src)}


def c_struct(src, name):
    m = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), src, re.S)
    assert m, name
    consts = _consts(src)
    out = []
    for decl in m.group(1).split(";"):
        decl = " ".join(decl.split())
        if not decl:
            continue
        m2 = re.match(r"(const\s+)?(\w+)\s*(\*?)\s*(.*)", decl)
        ctype, star, names = m2.group(2), m2.group(3), m2.group(4)
        for nm in names.split(","):
            nm = nm.strip()
            ptr = star or nm.startswith("*")
            nm = nm.lstrip("*").strip()
            arr = 1
            am = re.match(r"(\w+)\[(\w+)\]", nm)
            if am:
                nm, n = am.group(1), am.group(2)
                arr = int(n) if n.isdigit() else consts[n]
            out.append((nm, "ptr" if ptr else C_TYPES[ctype], arr))
    return out


def r_struct(src, name):
    m = re.search(r"pub struct %s \{(.*?)\}" % name, src, re.S)
    assert m, name
    out = []
    for fld in re.findall(r"pub\s+(\w+)\s*:\s*([^,]+?)\s*(?:,|$)", m.group(1).strip()):
        nm, ty = fld
        ty = ty.strip()
        if ty.startswith("*mut") or ty.startswith("*const"):
            out.append((nm, "ptr", 1))
            continue
        am = re.match(r"\[(\w+);\s*(\w+)\]", ty)
        if am:
            n = am.group(2)
            cm = re.search(r"pub const %s: usize = (\d+);" % n, src)
            out.append((nm, R_TYPES[am.group(1)], int(n) if n.isdigit() else int(cm.group(1))))
            continue
        out.append((nm, R_TYPES[ty], 1))
    return out


@pytest.mark.parametrize("name", STRUCTS)
def test_struct_layout_matches_header(name):
    src = open(LIBRS).read()
    assert re.search(r"#\[repr\(C\)\][^\n]*\n\s*pub struct %s\b" % name, src), "%s is not #[repr(C)]" % name
    assert r_struct(src, name) == c_struct(_header(), name)


def test_abi_version_and_constants():
    src = open(LIBRS).read()
    h = _header()
    consts = _consts(h)
    assert int(re.search(r"GS_ABI_VERSION: u32 = (\d+)", src).group(1)) == consts["GS_ABI_VERSION"]
    assert int(re.search(r"GS_HIST_BINS: usize = (\d+)", src).group(1)) == consts["GS_HIST_BINS"]
    assert int(re.search(r"GS_TRAFFIC_COLS: usize = (\d+)", src).group(1)) == int(
        re.search(r"GS_TRAFFIC_COLS\s*=\s*(\d+)", h).group(1))
    assert int(re.search(r"GS_COMM_ID_BYTES\s+(\d+)", h).group(1)) == int(
        re.search(r"internal: \[c_char; (\d+)\]", src).group(1))


def _c_functions(h):
    out = {}
    for m in re.finditer(r"\b(gs_[a-z_]+)\s*\(([^;{}]*?)\)\s*;", h):
        name, args = m.group(1), " ".join(m.group(2).split())
        if name in ("gs_block_fn",) or "(*" in m.group(0):
            continue
        out[name] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_extern_fns_match_header():
    src = open(LIBRS).read()
    ext = re.search(r'extern "C" \{(.*)\n\}', src, re.S).group(1)
    ext = re.sub(r"//[^\n]*", "", ext)
    rust = {}
    for m in re.finditer(r"pub fn (gs_\w+)\s*\(([^)]*)\)", ext):
        args = " ".join(m.group(2).split()).strip().rstrip(",")
        rust[m.group(1)] = 0 if not args else args.count(":")
    c = _c_functions(_header())
    assert set(rust) == set(c), (sorted(set(c) - set(rust)), sorted(set(rust) - set(c)))
    for k in c:
        assert rust[k] == c[k], (k, rust[k], c[k])


def test_cargo_manifest_and_build_script():
    d = os.path.join(ROOT, "rust", "gossipsim-sys")
    toml = open(os.path.join(d, "Cargo.toml")).read()
    assert 'name = "gossipsim-sys"' in toml and 'links = "gossipsim"' in toml
    b = open(os.path.join(d, "build.rs")).read()
    assert "rustc-link-lib=dylib=gossipsim" in b and "amdhip64" in b
