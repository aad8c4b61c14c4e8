"""The Rust binding (bindings/shadow-gpu-sys, the crate INTEGRATION.md §2 adds to Shadow as
src/lib/shadow-gpu-sys) against the C ABI it binds (include/shadow_gpu.h), mechanically.

No Rust toolchain is installed here, so the crate is not compiled; instead both files are
parsed and compared declaration by declaration:
  * every entry point of the header is declared in the crate's `extern "C"` block and vice
    versa, with the same argument count, argument types and return type (C -> Rust:
    int32_t i32, uint32_t u32, uint64_t u64, uint8_t u8, size_t usize, float f32, double
    f64, char c_char, void c_void; `const T*` *const T, `T*` *mut T, `T**` *mut *mut T) and
    the same argument names (Rust keywords renamed: `in` -> `input`);
  * every struct of the header is a #[repr(C)] struct in the crate with the same fields,
    in the same order, of the same types; every opaque handle is declared;
  * every #define and enum constant of the header has a crate constant of the same value;
  * every sg_* symbol the built library exports is declared in the header (and so in the
    crate): a function added to the library or the header without the crate fails here.
Reference conventions followed by the crate: the existing extern "C-unwind" exports of
/root/reference/src/main/core/worker.rs:619-684, the callers of graph/mod.rs:499-513.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "shadow_gpu.h")
CRATE = os.path.join(ROOT, "bindings", "shadow-gpu-sys")
LIB_RS = os.path.join(CRATE, "src", "lib.rs")
SO = os.path.join(ROOT, "shadow_amd", "libshadow_gpu.so")

CMAP = {"int32_t": "i32", "uint32_t": "u32", "uint64_t": "u64", "uint8_t": "u8", "uint16_t": "u16",
        "size_t": "usize", "float": "f32", "double": "f64", "char": "c_char", "void": "c_void"}
RUST_KEYWORDS = {"in": "input", "type": "ty", "fn": "func", "ref": "reference", "box": "boxed"}


# ---------------------------------------------------------------------------
# C header
# ---------------------------------------------------------------------------
def _strip_c(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _c_rust(base, stars):
    const = base.startswith("const ")
    t = CMAP.get(base.replace("const ", "").strip(), base.replace("const ", "").strip())
    for i in range(stars):
        t = f"*{'const' if const and i == 0 else 'mut'} {t}"
    return t


def parse_header(path):
    s = _strip_c(open(path).read())
    s = re.sub(r"#ifdef __cplusplus.*?#endif", " ", s, flags=re.S)
    consts = {k: int(v.rstrip("uU"), 0)
              for k, v in re.findall(r"#define\s+(SG_\w+)\s+(0x[0-9A-Fa-f]+[uU]?|\d+[uU]?)\s", s)}
    s = re.sub(r"#[^\n]*", " ", s)
    for body in re.findall(r"enum(?:\s+\w+)?\s*\{(.*?)\}", s, flags=re.S):
        consts.update({k: int(v) for k, v in re.findall(r"(SG_\w+)\s*=\s*(\d+)", body)})
    structs = {}
    for body, name in re.findall(r"typedef\s+struct\s+\w+\s*\{(.*?)\}\s*(\w+)\s*;", s, flags=re.S):
        fields = []
        for decl in body.split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            m = re.match(r"((?:const\s+)?\w+)\s*(.*)$", decl)
            for d in m.group(2).split(","):
                fields.append((d.replace("*", "").strip(), _c_rust(m.group(1), d.count("*"))))
        structs[name] = fields
    opaque = re.findall(r"typedef\s+struct\s+(\w+)\s+\1\s*;", s)
    body = re.sub(r"typedef\s+struct\s+\w+\s*\{.*?\}\s*\w+\s*;", " ", s, flags=re.S)
    body = re.sub(r"typedef[^;]*;", " ", body)
    body = re.sub(r"enum(?:\s+\w+)?\s*\{.*?\}\s*\w*\s*;", " ", body, flags=re.S)
    funcs = {}
    for ret, name, params in re.findall(r"((?:const\s+)?\w+\s*\**)\s*(sg_\w+)\s*\(([^)]*)\)\s*;", body):
        args = []
        params = " ".join(params.split())
        if params and params != "void":
            for p in params.split(","):
                m = re.match(r"((?:const\s+)?\w+)\s*(\**)\s*(\w+)$", p.strip())
                assert m, f"unparsed parameter {p!r} of {name}"
                args.append((m.group(3), _c_rust(m.group(1), len(m.group(2)))))
        r = " ".join(ret.split())
        rt = _c_rust(r.replace("*", "").strip(), r.count("*"))
        funcs[name] = (args, None if rt == "c_void" else rt)
    return dict(consts=consts, structs=structs, opaque=opaque, funcs=funcs)


# ---------------------------------------------------------------------------
# Rust crate
# ---------------------------------------------------------------------------
def _norm(t):
    return " ".join(t.replace("*const", "*const ").replace("*mut", "*mut ").split())


def parse_crate(path):
    s = re.sub(r"//[^\n]*", " ", open(path).read())  # comments and doc comments
    consts = {k: int(v.replace("_", ""), 0) for k, v in
              re.findall(r"pub\s+const\s+(SG_\w+)\s*:\s*\w+\s*=\s*(0x[0-9A-Fa-f_]+|\d[\d_]*)\s*;", s)}
    structs, opaque, repr_c = {}, [], set()
    for attrs, name, body in re.findall(r"((?:#\[[^\]]*\]\s*)*)pub\s+struct\s+(\w+)\s*\{(.*?)\}", s, flags=re.S):
        if "repr(C)" in attrs.replace(" ", ""):
            repr_c.add(name)
        fields = re.findall(r"pub\s+(\w+)\s*:\s*([^,]+),", body)
        if not fields and "_private" in body:
            opaque.append(name)
        else:
            structs[name] = [(f, _norm(t)) for f, t in fields]
    m = re.search(r'unsafe\s+extern\s+"C"\s*\{(.*)\}\s*$', s, flags=re.S)
    assert m, "no unsafe extern \"C\" block"
    funcs = {}
    for name, params, ret in re.findall(r"pub\s+fn\s+(\w+)\s*\(([^)]*)\)\s*(?:->\s*([^;]+))?;", m.group(1)):
        args = []
        for p in [x for x in " ".join(params.split()).split(",") if x.strip()]:
            n, t = p.split(":", 1)
            args.append((n.strip(), _norm(t)))
        funcs[name] = (args, _norm(ret) if ret.strip() else None)
    return dict(consts=consts, structs=structs, opaque=opaque, funcs=funcs, repr_c=repr_c)


@pytest.fixture(scope="module")
def both():
    return parse_header(HEADER), parse_crate(LIB_RS)


def test_crate_files_present():
    for f in ("Cargo.toml", "build.rs", os.path.join("src", "lib.rs")):
        assert os.path.isfile(os.path.join(CRATE, f)), f
    toml = open(os.path.join(CRATE, "Cargo.toml")).read()
    assert 'name = "shadow-gpu-sys"' in toml and 'links = "shadow_gpu"' in toml


def test_every_entry_point_matches(both):
    h, r = both
    assert len(h["funcs"]) >= 73
    missing = sorted(set(h["funcs"]) - set(r["funcs"]))
    extra = sorted(set(r["funcs"]) - set(h["funcs"]))
    assert not missing, f"declared in the header, not in the crate: {missing}"
    assert not extra, f"declared in the crate, not in the header: {extra}"
    for name, (cargs, cret) in h["funcs"].items():
        rargs, rret = r["funcs"][name]
        assert len(cargs) == len(rargs), f"{name}: {len(cargs)} C arguments, {len(rargs)} Rust"
        for (cn, ct), (rn, rt) in zip(cargs, rargs):
            assert RUST_KEYWORDS.get(cn, cn) == rn, f"{name}: argument {cn!r} is {rn!r} in the crate"
            assert _norm(ct) == rt, f"{name}({cn}): C {ct!r} vs Rust {rt!r}"
        assert (cret and _norm(cret)) == rret, f"{name}: returns C {cret!r} vs Rust {rret!r}"


def test_every_struct_matches(both):
    h, r = both
    assert set(h["opaque"]) == set(r["opaque"]), (h["opaque"], r["opaque"])
    assert set(h["structs"]) == set(r["structs"]), (sorted(h["structs"]), sorted(r["structs"]))
    for name, fields in h["structs"].items():
        assert name in r["repr_c"], f"{name} is not #[repr(C)]"
        got = r["structs"][name]
        assert [f for f, _ in fields] == [f for f, _ in got], f"{name}: field names/order differ"
        for (f, ct), (_, rt) in zip(fields, got):
            assert _norm(ct) == rt, f"{name}.{f}: C {ct!r} vs Rust {rt!r}"
    for name in h["opaque"]:
        assert name in r["repr_c"], f"{name} is not #[repr(C)]"


def test_every_constant_matches(both):
    h, r = both
    for k, v in h["consts"].items():
        assert k in r["consts"], f"constant {k} missing from the crate"
        assert r["consts"][k] == v, f"{k}: header {v}, crate {r['consts'][k]}"
    assert set(r["consts"]) == set(h["consts"]), sorted(set(r["consts"]) ^ set(h["consts"]))


def test_library_exports_are_declared(both):
    """Every sg_* function the built library exports is in the header (and hence the crate)."""
    h, _ = both
    if not os.path.exists(SO) or not shutil.which("nm"):
        pytest.skip("libshadow_gpu.so not built or nm missing")
    out = subprocess.run(["nm", "-D", "--defined-only", SO], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.split()[1:2] == ["T"] and ln.split()[-1].startswith("sg_")}
    assert exported == set(h["funcs"]), sorted(exported ^ set(h["funcs"]))


def test_checker_catches_drift(both, tmp_path):
    """The comparison is not vacuous: a crate with one argument's type changed, or one entry
    point dropped, fails it."""
    h, _ = both
    src = open(LIB_RS).read()
    bad = src.replace("pub fn sg_deliver_round(ctx: *mut sg_ctx, hosts: *mut sg_hosts, table: *const sg_table",
                      "pub fn sg_deliver_round(ctx: *mut sg_ctx, hosts: *const sg_hosts, table: *const sg_table")
    assert bad != src
    p = tmp_path / "lib.rs"
    p.write_text(bad)
    r = parse_crate(str(p))
    assert r["funcs"]["sg_deliver_round"][0][1][1] != _norm(h["funcs"]["sg_deliver_round"][0][1][1])
    p.write_text(re.sub(r"\n\s*pub fn sg_hosts_event_ctr[^;]*;", "\n", src))
    assert "sg_hosts_event_ctr" not in parse_crate(str(p))["funcs"]
