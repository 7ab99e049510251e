"""The Rust FFI crate (rust/merklekv-hip-sys) against the C header it binds (include/mkv_merkle.h): every
header function has exactly one `extern "C"` declaration with the same name, arity, parameter types
(pointer depth and constness at each level included) and return type, and the numeric #defines have Rust
constants of the same value. Rust is not installed in this image, so this is the check that the crate a
MerkleKV maintainer adds (sync.rs / server.rs call sites) matches the library;
the safe wrapper (src/merkle.rs) may only call functions the sys block declares."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "mkv_merkle.h")
CRATE = os.path.join(ROOT, "rust", "merklekv-hip-sys")

C_BASE = {"int": "c_int", "int32_t": "i32", "uint32_t": "u32", "uint64_t": "u64", "uint8_t": "u8", "double": "f64",
          "char": "c_char", "void": "c_void", "mkv_status": "mkv_status", "mkv_blob": "mkv_blob",
          "mkv_tree": "mkv_tree", "mkv_keylist": "mkv_keylist", "mkv_comm": "mkv_comm",
          "mkv_allgather_fn": "mkv_allgather_fn"}


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _c_type(decl, is_param=True):
    """'const mkv_tree *const *trees' -> ('mkv_tree', ['const', 'mut']) with the pointer levels listed
    outermost first, each as the constness of what that pointer points to (Rust's *const / *mut)."""
    decl = decl.strip()
    arr = False
    m = re.match(r"(.*?)\s*\[[^\]]*\]$", decl)
    if m:
        decl, arr = m.group(1), True
    toks = re.findall(r"\*|\w+", decl)
    if is_param:
        toks = toks[:-1]  # the parameter name
    base_const = False
    base = None
    quals = []  # constness of each pointer itself, innermost first
    for t in toks:
        if t == "*":
            quals.append(False)
        elif t == "const":
            if quals:
                quals[-1] = True
            else:
                base_const = True
        else:
            base = t
    pointee = [base_const] + quals[:-1] if quals else []
    levels = ["const" if c else "mut" for c in pointee]
    if arr:
        levels.append("const" if (quals[-1] if quals else base_const) else "mut")
    return C_BASE[base], levels[::-1]


def _rust_type(t):
    t = t.strip()
    levels = []
    while True:
        m = re.match(r"\*\s*(const|mut)\s+(.*)$", t)
        if not m:
            break
        levels.append(m.group(1))
        t = m.group(2).strip()
    return t, levels


def header_functions():
    s = _strip_c_comments(open(HDR).read())
    s = re.sub(r"\s+", " ", s)
    out = {}
    for ret, name, args in re.findall(r"(mkv_status|void|const char \*)\s*(mkv_\w+)\(([^()]*)\);", s):
        params = [] if args.strip() in ("", "void") else [_c_type(a) for a in args.split(",")]
        rt = {"mkv_status": ("mkv_status", []), "void": None, "const char *": ("c_char", ["const"])}[ret]
        assert name not in out, name
        out[name] = (params, rt)
    return out


def header_defines():
    out = {}
    for name, val in re.findall(r"#define (MKV_\w+) (\d+)\b", open(HDR).read()):
        out[name] = int(val)
    return out


def crate_functions():
    s = open(os.path.join(CRATE, "src", "lib.rs")).read()
    s = re.sub(r"//[^\n]*", " ", s)
    blocks = re.findall(r'extern "C" \{(.*?)\n\}', s, flags=re.S)
    assert len(blocks) == 1, "one extern \"C\" block"
    body = re.sub(r"\s+", " ", blocks[0])
    out = {}
    for name, args, ret in re.findall(r"pub fn (mkv_\w+)\((.*?)\)\s*(->\s*[^;]+)?;", body):
        params = []
        for a in [x for x in args.split(",") if x.strip()]:
            pname, ptype = a.split(":", 1)
            params.append(_rust_type(ptype))
        rt = _rust_type(ret[2:]) if ret else None
        assert name not in out, name
        out[name] = (params, rt)
    return out


def crate_consts():
    s = open(os.path.join(CRATE, "src", "lib.rs")).read()
    out = {}
    for name, expr in re.findall(r"pub const (MKV_\w+): \w+ = ([^;]+);", s):
        out[name] = expr.strip()
    return out


def test_every_header_function_is_declared_with_the_same_signature():
    h, r = header_functions(), crate_functions()
    assert len(h) >= 60
    assert set(h) == set(r), (sorted(set(h) - set(r)), sorted(set(r) - set(h)))
    for name, (params, ret) in h.items():
        rp, rr = r[name]
        assert len(params) == len(rp), name
        for i, (cp, rs) in enumerate(zip(params, rp)):
            assert cp == rs, (name, i, cp, rs)
        assert ret == rr, (name, ret, rr)


def test_numeric_defines_have_rust_constants():
    d, c = header_defines(), crate_consts()
    for name, v in d.items():
        assert name in c, name
        expr = c[name]
        val = eval(re.sub(r"MKV_\w+", lambda m: str(d.get(m.group(0), c.get(m.group(0)))), expr))
        assert val == v, (name, val, v)
    assert eval(c["MKV_FRINGE_BYTES"].replace("MKV_FRINGE_ENTRY_BYTES", str(d["MKV_FRINGE_ENTRY_BYTES"]))
                .replace("MKV_FRINGE_MAX_ENTRIES", str(d["MKV_FRINGE_MAX_ENTRIES"]))) == \
        d["MKV_FRINGE_ENTRY_BYTES"] * d["MKV_FRINGE_MAX_ENTRIES"]


def test_safe_wrapper_calls_only_declared_functions_and_keeps_reference_api():
    r = crate_functions()
    src = open(os.path.join(CRATE, "src", "merkle.rs")).read()
    called = set(re.findall(r"\b(mkv_\w+)\(", src))
    assert called and called <= set(r), sorted(called - set(r))
    # the reference's public surface (merkle.rs:36-204) with its receivers
    for sig in ("pub fn new() -> Self", "pub fn insert(&mut self, key: &str, value: &str)",
                "pub fn remove(&mut self, key: &str)", "pub fn get_root_hash(&self) -> Option<&Vec<u8>>",
                "pub fn diff_keys(&self, other: &MerkleTree) -> Vec<String>",
                "pub fn diff_first_key(&self, other: &MerkleTree) -> Option<String>",
                "pub fn inorder_keys(&self) -> Vec<String>", "pub fn leaves(&self) -> Vec<(String, Vec<u8>)>",
                "pub fn node_count(&self) -> usize", "impl Clone for MerkleTree", "impl std::fmt::Debug for MerkleTree"):
        assert sig in src, sig


def test_crate_manifest_links_the_library():
    toml = open(os.path.join(CRATE, "Cargo.toml")).read()
    assert 'links = "merklekv_hip"' in toml
    b = open(os.path.join(CRATE, "build.rs")).read()
    assert "rustc-link-lib=dylib=merklekv_hip" in b and "merklekv_amd/lib" in b
