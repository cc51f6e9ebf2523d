"""CPU: the Rust binding (bindings/rust) against the C ABI it binds.

There is no Rust toolchain in this image, so the binding cannot be compiled here.
This test does the checks a compiler would make at the boundary:
  - every `extern "C"` function in bindings/rust/**/*.rs is declared in
    include/iris_hip.h with the same name, the same number of arguments and the
    same C types (pointer depth and pointee constness included), the same return
    type; and every function of the header has a Rust declaration;
  - the #[repr(C)] structs and the constants equal the header's;
  - the drop-in items keep the reference signatures (src/arch/generic.rs:4,11,
    src/lib.rs:33,42,60,69,82,89);
  - the reference-crate patch applies to the reference sources when they are present;
  - the Rust sources are bracket-balanced (a cheap syntax sanity check)."""
import pathlib
import re
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
RUST = ROOT / "bindings" / "rust"
HEADER = ROOT / "include" / "iris_hip.h"

C_BASE = {"void", "char", "int", "double", "size_t", "uint8_t", "uint16_t", "uint32_t", "uint64_t", "int32_t",
          "iris_device_t", "iris_db_t", "iris_engine_t", "iris_pending_t", "iris_match_t", "iris_template_t",
          "iris_group_t", "iris_group_db_t", "iris_group_pending_t"}
RUST_TO_C = {"c_void": "void", "c_char": "char", "c_int": "int", "f64": "double", "usize": "size_t", "u8": "uint8_t",
             "u16": "uint16_t", "u32": "uint32_t", "u64": "uint64_t", "i32": "int32_t", "IrisDevice": "iris_device_t",
             "IrisDb": "iris_db_t", "IrisEngine": "iris_engine_t", "IrisPending": "iris_pending_t",
             "IrisMatch": "iris_match_t", "IrisTemplate": "iris_template_t", "IrisGroup": "iris_group_t",
             "IrisGroupDb": "iris_group_db_t", "IrisGroupPending": "iris_group_pending_t"}


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def c_type(decl, has_name=True):
    """Canonical (base, (pointee-const flags from the innermost outwards)) of a C
    parameter / return declaration; array parameters decay to pointers."""
    decl = decl.strip()
    arrays = 0
    m = re.search(r"(\[[^\]]*\])+\s*$", decl)
    if m:
        arrays = m.group(0).count("[")
        decl = decl[:m.start()].strip()
    toks = re.findall(r"\*|[A-Za-z_]\w*", decl)
    if has_name and toks and toks[-1] not in ("*", "const") and toks[-1] not in C_BASE:
        toks = toks[:-1]  # the parameter name
    base, base_const, ptrs = None, False, []
    for t in toks:
        if t == "const":
            if ptrs:
                ptrs[-1] = True
            else:
                base_const = True
        elif t == "*":
            ptrs.append(False)
        else:
            assert base is None, decl
            base = t
    assert base in C_BASE, f"unknown C type in {decl!r}"
    # constness of the object at each level, innermost (the base) first; the outermost
    # pointer's own qualifier is top-level and does not change the type seen by the callee
    depth = len(ptrs) + arrays
    consts = [base_const] + ptrs
    return base, tuple(consts[:depth]), depth


def rust_type(t):
    t = t.strip()
    flags = []
    depth = 0
    while t.startswith("*"):
        m = re.match(r"\*(const|mut)\s+", t)
        assert m, t
        flags.append(m.group(1) == "const")
        t = t[m.end():]
        depth += 1
    arr = re.fullmatch(r"\[\s*(\w+)\s*;\s*\w+\s*\]", t)
    if arr:
        assert depth >= 1, f"array by value: {t}"
        t = arr.group(1)
    assert t in RUST_TO_C, f"unknown Rust FFI type {t!r}"
    # flags were collected outermost first: pointee constness of each level
    return RUST_TO_C[t], tuple(reversed(flags)), depth


def header_functions():
    src = _strip_c_comments(HEADER.read_text())
    src = re.sub(r"^\s*#.*$", " ", src, flags=re.M)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(iris_\w+)\s*\(([^)]*)\)\s*;", src):
        ret, name, params = m.group(1), m.group(2), m.group(3).strip()
        ret = ret.replace("extern", "").strip()
        args = [] if params in ("", "void") else [c_type(p) for p in params.split(",")]
        out[name] = (c_type(ret, has_name=False), args)
    return out


def rust_extern_functions():
    out = {}
    for path in sorted(RUST.rglob("*.rs")):
        text = re.sub(r"//[^\n]*", "", path.read_text())
        for blk in re.finditer(r'extern\s+"C"\s*\{', text):
            i, depth = blk.end(), 1
            while depth:
                depth += {"{": 1, "}": -1}.get(text[i], 0)
                i += 1
            body = text[blk.end():i - 1]
            for fm in re.finditer(r"(?:pub\s+)?fn\s+(\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+))?;", body, flags=re.S):
                name, params, ret = fm.group(1), fm.group(2), fm.group(3)
                args = []
                for p in [p for p in _split_top(params) if p.strip()]:
                    pname, ptype = p.split(":", 1)
                    args.append(rust_type(ptype))
                assert name not in out, f"{name} declared twice"
                out[name] = (rust_type(ret) if ret else ("void", (), 0), args, path.relative_to(ROOT))
    return out


def _split_top(s):
    parts, depth, cur = [], 0, ""
    for ch in s:
        if ch in "[(<":
            depth += 1
        elif ch in "])>":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    parts.append(cur)
    return parts


def test_c_type_canonicalisation():
    assert c_type("const uint16_t *const *shares") == ("uint16_t", (True, True), 2)
    assert c_type("iris_db_t *const *shares") == ("iris_db_t", (False, True), 2)
    assert c_type("const uint8_t key[32]") == ("uint8_t", (True,), 1)
    assert c_type("uint64_t out[IRIS_LIMBS]") == ("uint64_t", (False,), 1)
    assert c_type("iris_device_t **out") == ("iris_device_t", (False, False), 2)
    assert c_type("uint64_t n") == ("uint64_t", (), 0)
    assert rust_type("*const *const u16") == ("uint16_t", (True, True), 2)
    assert rust_type("*const *mut IrisDb") == ("iris_db_t", (False, True), 2)
    assert rust_type("*const [u8; 32]") == ("uint8_t", (True,), 1)
    assert rust_type("*mut *mut IrisDevice") == ("iris_device_t", (False, False), 2)


def test_extern_blocks_match_header():
    hdr = header_functions()
    rs = rust_extern_functions()
    assert len(hdr) >= 60
    missing = sorted(set(hdr) - set(rs))
    assert not missing, f"header functions without a Rust declaration: {missing}"
    for name, (ret, args, path) in rs.items():
        assert name in hdr, f"{path}: {name} is not in include/iris_hip.h"
        hret, hargs = hdr[name]
        assert len(args) == len(hargs), f"{name}: {len(args)} Rust args, {len(hargs)} in the header"
        assert ret == hret, f"{name}: return {ret} vs {hret}"
        for k, (a, h) in enumerate(zip(args, hargs)):
            assert a == h, f"{name} arg {k}: Rust {a} vs C {h}"


def _header_struct(name):
    src = _strip_c_comments(HEADER.read_text())
    m = re.search(r"typedef struct \w+ \{([^{}]*)\}\s*" + name + r"\s*;", src)
    fields = []
    for decl in m.group(1).split(";"):
        decl = decl.strip()
        if decl:
            arr = re.search(r"\[(\w+)\]$", decl)
            toks = re.findall(r"\w+", re.sub(r"\[.*\]", "", decl))
            fields.append((toks[-1], toks[-2], arr.group(1) if arr else None))
    return fields


def _rust_struct(name):
    text = (RUST / "src" / "iris_hip" / "ffi.rs").read_text()
    m = re.search(r"pub struct " + name + r"\s*\{(.*?)\}", text, flags=re.S)
    fields = []
    for f in re.finditer(r"pub (\w+):\s*([^,]+),", m.group(1)):
        t = f.group(2).strip()
        arr = re.fullmatch(r"\[(\w+);\s*(\w+)\]", t)
        fields.append((f.group(1), RUST_TO_C[arr.group(1) if arr else t], arr.group(2) if arr else None))
    return fields


def test_structs_and_constants_match():
    assert _rust_struct("IrisMatch") == _header_struct("iris_match_t")
    assert [(n, t) for n, t, _ in _rust_struct("IrisTemplate")] == [(n, t) for n, t, _ in
                                                                    _header_struct("iris_template_t")]
    hdr_defs = dict(re.findall(r"#define (IRIS_\w+) \(?(-?\d+)\)?", HEADER.read_text()))
    rs_defs = dict(re.findall(r"pub const (IRIS_\w+): \w+ = (-?\d+);", (RUST / "src/iris_hip/ffi.rs").read_text()))
    assert hdr_defs and set(hdr_defs) == set(rs_defs)
    for k, v in hdr_defs.items():
        assert int(rs_defs[k]) == int(v), k


def test_reference_signatures_kept():
    hip = (RUST / "src" / "arch" / "hip.rs").read_text()
    assert re.search(r"pub fn dot_bool\(a: &\[u64; LIMBS\], b: &\[u64; LIMBS\]\) -> u16", hip)
    assert re.search(r"pub fn dot_u16\(a: &\[u16; BITS\], b: &\[u16; BITS\]\) -> u16", hip)
    eng = (RUST / "src" / "iris_hip" / "engines.rs").read_text()
    for sig in [r"impl DistanceEngine \{\s*pub fn new\(query: &EncodedBits\) -> Self",
                r"impl MasksEngine \{\s*pub fn new\(query: &Bits\) -> Self",
                r"pub fn batch_process\(&self, out: &mut \[\[u16; 31\]\], db: &\[EncodedBits\]\)",
                r"pub fn batch_process\(&self, out: &mut \[\[u16; 31\]\], db: &\[Bits\]\)",
                r"pub fn distances\(query: &EncodedBits, entry: &EncodedBits\) -> \[u16; 31\]",
                r"pub fn denominators\(query: &Bits, entry: &Bits\) -> \[u16; 31\]"]:
        assert re.search(sig, eng), sig
    # no `?` on a function returning () and no undeclared handle types in the docs' snippets
    doc = (ROOT / "INTEGRATION.md").read_text()
    assert "new_on(dev, q)" not in doc


def test_rust_sources_balanced():
    for path in RUST.rglob("*.rs"):
        text = path.read_text()
        text = re.sub(r"//[^\n]*", "", text)
        text = re.sub(r'"(?:\\.|[^"\\])*"', '""', text)
        text = re.sub(r"'(?:\\.|[^'\\])'", "''", text)
        for o, c in ("{}", "()", "[]"):
            assert text.count(o) == text.count(c), f"{path}: unbalanced {o}{c}"


@pytest.mark.skipif(not pathlib.Path("/root/reference/src/lib.rs").exists() or shutil.which("patch") is None,
                    reason="reference sources not present (GPU box)")
def test_reference_patch_applies(tmp_path):
    for name in ("src", "Cargo.toml", "build.rs"):
        src = pathlib.Path("/root/reference") / name
        (shutil.copytree if src.is_dir() else shutil.copy)(src, tmp_path / name)
    r = subprocess.run(["patch", "-p1", "--dry-run", "-i", str(RUST / "reference.patch")], cwd=tmp_path,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.skipif(not pathlib.Path("/root/reference/src/lib.rs").exists(),
                    reason="reference sources not present (GPU box)")
def test_reference_items_the_binding_relies_on():
    """Textual checks of the reference items bindings/rust uses (what rustc would check):
    crate-visible LIMBS (arch/hip.rs), public tuple fields of Bits / EncodedBits
    (engines.rs passes query.0), a Copy Template (TemplateEngine keeps its query), and the
    exact `pub use` / struct lines reference.patch rewrites."""
    ref = pathlib.Path("/root/reference/src")
    bits = (ref / "bits.rs").read_text()
    assert re.search(r"pub(\(crate\))? const LIMBS: usize", bits)
    assert "pub struct Bits(pub [u64; LIMBS]);" in bits
    assert re.search(r"pub struct EncodedBits\(pub \[u16; BITS\]\);", (ref / "encoded_bits.rs").read_text())
    tmpl = (ref / "template.rs").read_text()
    derive = re.search(r"#\[derive\(([^)]*)\)\]\s*pub struct Template", tmpl, flags=re.S)
    assert derive and re.search(r"\bCopy\b", derive.group(1))
    assert "pub use generic::{dot_bool, dot_u16};" in (ref / "arch" / "mod.rs").read_text()
    lib = (ref / "lib.rs").read_text()
    for line in ("pub use crate::{bits::Bits, encoded_bits::EncodedBits, template::Template};",
                 "pub struct DistanceEngine {", "pub struct MasksEngine {", "impl DistanceEngine {",
                 "impl MasksEngine {", "mod template;"):
        assert line in lib, line
    patch = (RUST / "reference.patch").read_text()
    assert "+pub use hip::{dot_bool, dot_u16};" in patch and "+pub use iris_hip::engines::{DistanceEngine, MasksEngine};" in patch
